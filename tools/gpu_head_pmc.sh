#!/bin/bash
# cv_head L2 behaviour: TCC hit / miss, TCP accesses (separate passes), averaged over cv_head launches
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-hpmc}; mkdir -p $OUT; export TMPDIR=/tmp
for pass in "TCC_HIT_sum TCC_MISS_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "TA_BUSY_avr TA_TA_BUSY_sum" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAIT_ANY"; do
  timeout -s KILL 90 rocprofv3 --pmc $pass -d $GRAFT_REPO_ROOT/$OUT/pmc -o p --output-format csv -- python3 tools/hip_reg_layers.py --only cv_head --reps 3 > $OUT/pmc_run.log 2>&1; echo "pass [$pass] rc=$?"
  python3 - <<'PY' "$OUT"
import csv, glob, sys, collections
out = sys.argv[1]
rows = []
for f in glob.glob(out + "/pmc/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(list)
for r in rows:
    if "cv_head_kernel" in r.get("Kernel_Name", ""):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print("  %-32s %.4g (n=%d)" % (k, sum(v) / len(v), len(v)))
PY
  rm -rf $OUT/pmc
done
