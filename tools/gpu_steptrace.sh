#!/bin/bash
# eval step: kernel trace (one step's sequence with gaps) and three 50-rep timings
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-st}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$OUT/tr" -o run --output-format csv -- \
  python3 tools/hip_reg_layers.py --only step --reps 10 > $OUT/tr.log 2>&1; echo "trace rc=$?"
for i in 1 2 3; do timeout -k 10 240 python -u tools/hip_reg_layers.py --only step --reps 50 2>&1 | grep -E "ms$"; done
