#!/bin/bash
# rocprof kernel trace of the fused op alone (bench --kernel-only): prologue / fold / main kernel durations
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r3w}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --kernel-only > $OUT/b.json 2> $OUT/b.err; rc=$?; echo "prof rc=$rc"
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/*/prof/run_kernel_trace.csv")
f = [x for x in f if "r3w" in x][0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    d[(r["Kernel_Name"][:70], r["Grid_Size_X"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:14]:
    print("%8.1f us x%3d  %s grid %s" % (sum(v) / len(v) / 1e3, len(v), k[0], k[1]))
PY
exit $rc
