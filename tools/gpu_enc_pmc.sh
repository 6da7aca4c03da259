#!/bin/bash
# conv2d: GPU parity tests, eval-step time, and two PMC passes over tools/enc_layers.py
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-encp}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k conv2d > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $OUT/pytest.log | head; exit $rc; }
timeout -k 10 240 python -u tools/hip_reg_layers.py --only step --reps 20 2>&1 | grep -E "ms$"
timeout -k 10 240 python -u tools/enc_layers.py --reps 10 2>&1 | grep -v amdgpu.ids
n=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F32"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass -d $GRAFT_REPO_ROOT/$OUT/pmc$n -o p --output-format csv -- python3 tools/enc_layers.py --reps 2 > $OUT/pmc_run$n.log 2>&1; echo "pmc$n rc=$?"
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "conv2d_narrow" not in k: continue
        k = k[k.index("kernel<") + 7:k.index(">")]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, " ".join("%s=%.3g" % (c.replace("SQ_", ""), sum(v) / len(v)) for c, v in sorted(d.items())))
PY
