#!/bin/bash
# cv_head ablations: time the fused kernel with parts removed (results discarded), then PMC of the real one
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-abl}; mkdir -p $OUT; export TMPDIR=/tmp
for v in ${VARIANTS:-default ablp ablc ablpc}; do
  if [ $v != default ]; then L=$GRAFT_REPO_ROOT/tools/exp_libs/lib$v.so; else L=; fi
  echo "== $v"; MVS_LIB_PATH=$L timeout -k 10 200 python -u tools/hip_reg_layers.py --only cv_head,cv_split --reps 10 2>&1 | grep -E "^cv_" || exit 1
done
[ -n "$NOPMC" ] && exit 0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"; do
  timeout -s KILL 90 rocprofv3 --pmc $pass -d $GRAFT_REPO_ROOT/$OUT/pmc -o p --output-format csv -- python3 tools/hip_reg_layers.py --only cv_head --reps 3 > $OUT/pmc_run.log 2>&1; echo "pmc rc=$?"
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
    print("%-28s %.4g (n=%d)" % (k, sum(v) / len(v), len(v)))
PY
  rm -rf $OUT/pmc
done
