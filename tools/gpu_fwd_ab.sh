# A/B timing of fused-forward library variants (tools/exp_libs/lib*.so), channel-quad store, cfg 2/3/5
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; export MVS_BENCH_C4=1
for v in "$@"; do
  echo "== $v"
  MVS_LIB_PATH="$GRAFT_REPO_ROOT/tools/exp_libs/lib$v.so" timeout -k 10 200 python3 -u tools/kernel_bench.py 2 3 5 2>&1 | grep cfg || exit 1
done
