# conv2d kernel parity + end-to-end tests, then the eval / train-mode step timings
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "conv2d or end_to_end or live or deconv or train_mode or narrow" > gpurun_out/conv2d_tests.log 2>&1; rc=$?; tail -15 gpurun_out/conv2d_tests.log; [ $rc -ne 0 ] && exit $rc
for m in eval train; do timeout -k 10 200 python3 -u tools/step_trace.py --mode $m 2>&1 | grep "step:" || exit 1; done
