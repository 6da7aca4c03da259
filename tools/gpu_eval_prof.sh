# kernel-trace stats of the eval step (tools/step_trace.py) -> gpurun_out/<tag>_eval/
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-cur}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${T}_eval" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/step_trace.py" --mode eval > gpurun_out/${T}_eval.log 2>&1; rc=$?; echo "eval prof rc=$rc"; grep "step:" gpurun_out/${T}_eval.log
exit $rc
