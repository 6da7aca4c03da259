# train-mode BN kernels + live path tests, train step profile, forward prefetch A/B
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -rf --timeout 300 --timeout-method thread -k "train_mode or end_to_end or channel_stats" > gpurun_out/r2i_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r2i_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r2i_train" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/step_trace.py" --mode train > gpurun_out/r2i_train.log 2>&1; rc=$?; echo "train prof rc=$rc"; grep "step:" gpurun_out/r2i_train.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_fwd_ab.sh U F1 U F1
