# GPU: selected tests (TESTS, default all -m gpu) then kernel bench; each step time-limited.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -v -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | tail -8
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/kernel_bench.py > gpurun_out/kernel_bench.log 2>&1; rc=$?; echo "kbench rc=$rc"; cat gpurun_out/kernel_bench.log | grep cfg
exit $rc
