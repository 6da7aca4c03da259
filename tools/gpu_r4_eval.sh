#!/bin/bash
# round 4: eval-step kernel trace (the bench step alone) + per-layer times
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-r4e}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/eval" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/step_trace.py" --mode ${MODE:-eval} > $OUT/eval.log 2>&1; rc=$?; echo "eval prof rc=$rc"; grep "step:" $OUT/eval.log
python3 - $OUT/eval/run_kernel_stats.csv <<'PY'
import csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(x['TotalDurationNs']) for x in r)
n = 13
for x in r[:26]:
    print('%7.3f ms/step %4s calls  %s' % (float(x['TotalDurationNs']) / 1e6 / n, x['Calls'], x['Name'][:100]))
print('total %.3f ms/step' % (tot / 1e6 / n))
PY
exit $rc
