# Round 2: new config parity tests + atomics microbenchmark
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o /tmp/atomic_patterns tools/microbench/atomic_patterns.hip || exit 1
timeout -k 10 120 /tmp/atomic_patterns > gpurun_out/atomic_patterns.log 2>&1; rc=$?; cat gpurun_out/atomic_patterns.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -v -rf --timeout 300 --timeout-method thread > gpurun_out/r2b_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/r2b_pytest.log
exit $rc
