# forward parity tests on the in-tree library, then A/B of fused-forward variants (all configs)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_bf16_cost_volume.py -m gpu > gpurun_out/fwd_tests.log 2>&1 || { tail -30 gpurun_out/fwd_tests.log; exit 1; }
tail -3 gpurun_out/fwd_tests.log
for v in "$@"; do
  echo "== $v"
  MVS_LIB_PATH="$GRAFT_REPO_ROOT/tools/exp_libs/lib$v.so" MVS_BENCH_C4=1 timeout -k 10 200 python3 -u tools/kernel_bench.py 2 3 5 2>&1 | grep cfg || exit 1
  MVS_LIB_PATH="$GRAFT_REPO_ROOT/tools/exp_libs/lib$v.so" timeout -k 10 200 python3 -u tools/kernel_bench.py 4 2>&1 | grep cfg || exit 1
done
