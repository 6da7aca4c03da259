# A/B timing of backward library variants (tools/exp_libs/lib*.so) at cfg 1/2/3
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "$@"; do
  echo "== $v"
  MVS_LIB_PATH="$GRAFT_REPO_ROOT/tools/exp_libs/lib$v.so" timeout -k 10 200 python3 -u tools/bwd_bench.py 1 2 3 2>&1 | grep cfg || exit 1
done
