# A/B per-layer times of library variants (tools/exp_libs/lib<name>.so) at cfg 2:
#   bash tools/gpu_layer_ab.sh <layers,comma,separated> <variant> [<variant> ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
layers=$1; shift
for v in "$@"; do
  echo "== $v"
  MVS_LIB_PATH="$PWD/tools/exp_libs/lib$v.so" timeout -k 10 150 python3 -u tools/hip_reg_layers.py --only "$layers" --reps 20 2>&1 | grep -E "ms$|rror" || exit $?
done
