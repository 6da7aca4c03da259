# A/B of library variants on the eval and train-mode steps (tools/step_trace.py)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "$@"; do
  for m in eval train; do
    MVS_LIB_PATH="$GRAFT_REPO_ROOT/tools/exp_libs/lib$v.so" timeout -k 10 200 python3 -u tools/step_trace.py --mode $m 2>&1 | grep "step:" | sed "s/^/$v /" || exit 1
  done
done
