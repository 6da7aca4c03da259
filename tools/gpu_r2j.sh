# forward staging change: full GPU parity + config tests
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/r2j_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r2j_pytest.log
exit $rc
