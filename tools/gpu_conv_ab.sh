# A/B timing of conv3d_k3 library variants (tools/exp_libs/lib*.so) at the cfg2 shape
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "$@"; do
  echo "== $v"
  MVS_LIB_PATH="$GRAFT_REPO_ROOT/tools/exp_libs/lib$v.so" timeout -k 10 120 python3 -u tools/conv_bench.py 20 || exit $?
done
