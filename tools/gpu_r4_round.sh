#!/bin/bash
# round 4: full GPU suite (+ parity records), smoke, bench (N=1), rocprof kernel trace of a short bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-r4r}; mkdir -p $OUT; export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
MVS_PARITY_OUT=$OUT/parity timeout -k 10 1100 python -u -m pytest tests -m gpu -v -rf --timeout 600 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head; tail -2 $OUT/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 $OUT/smoke.log
fi
s=$(date +%s); timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc wall=$(( $(date +%s) - s ))s"
if [ $rc -ne 0 ]; then tail -20 $OUT/bench.err; exit $rc; fi
python3 - $OUT/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("value %.1f maps/s, %.3f ms/step; head %.3f ms, %.1f TF/s f16 exec (frac %.3f), fp32-conv %.1f TF/s, hbm %.0f GB/s" % (
    d["value"], d["ms_per_step"], r["kernel_ms"], r["achieved"], r["frac"], r.get("alg_fp32_conv_tflops", 0), r.get("hbm_GBps", 0)))
print("exact_fp32 %s; warp kernel %.3f ms frac %.3f; bwd %s; train_bn %s; train_step %s" % (d.get("exact_fp32_step", {}).get("ms_per_step"),
    d["warp_kernel"]["kernel_ms"], d["warp_kernel"]["frac"], d["cost_volume_backward"].get("bwd_ms"), d.get("train_bn", {}).get("ms_per_step"),
    d.get("train_step", {}).get("ms_per_step")))
PY
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra --no-train-step > $OUT/prof_bench.json 2> $OUT/prof_bench.err; echo "prof rc=$?"
f=$(ls $OUT/prof/*/run_kernel_stats.csv $OUT/prof/run_kernel_stats.csv 2>/dev/null | head -1); head -12 "$f" | cut -c1-150
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/proft" -o run --output-format csv -- \
  python3 tools/train_step_prof.py > $OUT/prof_train.log 2>&1; echo "train prof rc=$?"; tail -1 $OUT/prof_train.log
f=$(ls $OUT/proft/*/run_kernel_stats.csv $OUT/proft/run_kernel_stats.csv 2>/dev/null | head -1); head -6 "$f" | cut -c1-150
