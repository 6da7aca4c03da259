#!/bin/bash
# Round 4 baseline: per-layer times and the eval-step kernel trace of the round-3 tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r4a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/hip_reg_layers.py > $OUT/reg_layers.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/reg_layers.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/eval" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/step_trace.py" --mode eval > $OUT/eval.log 2>&1; rc=$?; echo "eval prof rc=$rc"; grep "step:" $OUT/eval.log
exit $rc
