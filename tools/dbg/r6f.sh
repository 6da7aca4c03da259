cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/r6f; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 -k "pipelined or s1_lds or region_conv_matches" > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for c in 1 2 4; do
MVS_PIPELINE_CHUNKS=$c timeout -k 10 300 python -u tools/fp32_layers.py --only step,step --reps 30 > $OUT/step_c$c.log 2>&1; rc=$?; echo "chunks $c rc=$rc"; grep step $OUT/step_c$c.log; [ $rc -ne 0 ] && exit $rc
done
MVS_ARITHMETIC=split_f16 MVS_PIPELINE_CHUNKS=2 timeout -k 10 300 python -u tools/step_trace.py --arithmetic split_f16 --steps 20 > $OUT/split_c2.log 2>&1; echo "split c2 rc=$?"; cat $OUT/split_c2.log | grep step
MVS_PIPELINE_CHUNKS=1 timeout -k 10 300 python -u tools/step_trace.py --arithmetic split_f16 --steps 20 > $OUT/split_c1.log 2>&1; echo "split c1 rc=$?"; cat $OUT/split_c1.log | grep step
exit 0
