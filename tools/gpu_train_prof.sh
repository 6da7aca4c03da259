# kernel-trace stats of the train-mode-BN step (tools/step_trace.py --mode train) -> gpurun_out/<tag>_train/
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-cur}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${T}_train" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/step_trace.py" --mode train > gpurun_out/${T}_train.log 2>&1; rc=$?; echo "train prof rc=$rc"; grep "step:" gpurun_out/${T}_train.log
exit $rc
