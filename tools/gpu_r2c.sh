# Round 2: backward rewrite -- parity tests, timing, rocprof stats; then the cfg-2 e2e parity test
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -rf --timeout 200 --timeout-method thread -k "backward or smoke" > gpurun_out/r2c_pytest_bwd.log 2>&1; rc=$?; echo "pytest bwd rc=$rc"; tail -15 gpurun_out/r2c_pytest_bwd.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bwd_bench.py > gpurun_out/r2c_bwd_bench.log 2>&1; rc=$?; echo "bwd bench rc=$rc"; grep cfg gpurun_out/r2c_bwd_bench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r2c_bwd_prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/bwd_bench.py" 2 > gpurun_out/r2c_bwd_prof.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -rf --timeout 300 --timeout-method thread -k "cfg2" > gpurun_out/r2c_pytest_cfg2.log 2>&1; rc=$?; echo "pytest cfg2 rc=$rc"; tail -15 gpurun_out/r2c_pytest_cfg2.log
exit $rc
