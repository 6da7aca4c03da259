# round-3 A/B of backward variants (tools/exp_libs/lib*.so) after the backward parity tests
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "backward or golden" > gpurun_out/bwd_tests.log 2>&1 || { tail -30 gpurun_out/bwd_tests.log; exit 1; }
tail -3 gpurun_out/bwd_tests.log
bash tools/gpu_bwd_ab.sh "$@"
