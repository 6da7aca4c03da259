cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bf16_cost_volume.py -m gpu -v -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | tail -8
if [ $rc -gt 1 ]; then exit $rc; fi
MVS_BENCH_BF16=1 timeout -k 10 200 python tools/kernel_bench.py 2 3 5 > gpurun_out/kb16.log 2>&1; rc=$?
echo "kbench rc=$rc"; grep cfg gpurun_out/kb16.log | cut -c1-190
exit $rc
