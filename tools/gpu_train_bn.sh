# train-mode BN live path: GPU parity tests + the e2e tests (train mode) + the bench's train_bn leg
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -rf --timeout 300 --timeout-method thread -k "train_mode or end_to_end" > gpurun_out/trbn_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/trbn_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/trbn_prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/step_trace.py" --mode train > gpurun_out/trbn_step.log 2>&1; rc=$?; echo "train prof rc=$rc"; grep "step:" gpurun_out/trbn_step.log
exit $rc
