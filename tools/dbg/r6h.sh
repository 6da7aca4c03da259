cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/r6h; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 -k "rccl or pipelined or sharded" > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error" $OUT/pytest.log | head; tail -3 $OUT/pytest.log
for v in 2 4; do
MVS_S2_RB=$v timeout -k 10 300 python -u tools/fp32_layers.py --only conv_1_0,conv_2_0,step,step --reps 30 > $OUT/s2rb$v.log 2>&1; echo "s2 rb $v rc=$?"; grep ms $OUT/s2rb$v.log
done
exit 0
