# Round 2: channel-quad cost-volume feed -- parity, end-to-end parity, step profile
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -rf --timeout 200 --timeout-method thread -k "quad or region or regulariser or end_to_end or conv or golden" > gpurun_out/r2h_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/r2h_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r2h_eval" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/step_trace.py" --mode eval > gpurun_out/r2h_eval.log 2>&1; rc=$?; echo "eval prof rc=$rc"; grep "step:" gpurun_out/r2h_eval.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -rf --timeout 300 --timeout-method thread -k "cfg2" > gpurun_out/r2h_pytest_cfg2.log 2>&1; rc=$?; echo "pytest cfg2 rc=$rc"; tail -5 gpurun_out/r2h_pytest_cfg2.log
exit $rc
