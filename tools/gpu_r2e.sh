# Round 2: backward (view subsets) + packed-FMA conv_0_0: parity tests, timings, profiles
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -rf --timeout 200 --timeout-method thread -k "backward or conv or regulariser or deconv or end_to_end" > gpurun_out/r2e_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/r2e_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bwd_bench.py > gpurun_out/r2e_bwd_bench.log 2>&1; rc=$?; echo "bwd bench rc=$rc"; grep cfg gpurun_out/r2e_bwd_bench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r2e_eval" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/step_trace.py" --mode eval > gpurun_out/r2e_eval.log 2>&1; rc=$?; echo "eval prof rc=$rc"; grep "step:" gpurun_out/r2e_eval.log
exit $rc
