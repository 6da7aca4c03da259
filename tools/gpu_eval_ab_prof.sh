# A/B of library variants: per-kernel eval-step times (rocprofv3 kernel-trace stats per variant)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "$@"; do
  MVS_LIB_PATH="$GRAFT_REPO_ROOT/tools/exp_libs/lib$v.so" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/ab_$v" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/step_trace.py" --mode eval > gpurun_out/ab_$v.log 2>&1 || exit 1
  grep "step:" gpurun_out/ab_$v.log | sed "s/^/$v /"
done
