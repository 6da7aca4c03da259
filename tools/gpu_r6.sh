#!/bin/bash
# round 6 GPU driver: bash tools/gpu_r6.sh <tag> [stages...]   stages: tests smoke bench prof cfgprof evalprof pmc
#   (default: tests smoke bench prof pmc)
#   tests  full GPU suite (+ parity records under $OUT/parity)
#   smoke  __graft_entry__.smoke()
#   bench  python bench.py (N=1 defaults) -> $OUT/bench.json
#   prof   rocprofv3 --kernel-trace --stats of a short bench (the roofline agreement source)
#   pmc    head counters, one counter group per rocprofv3 pass, on tools/hip_reg_layers.py --only cv_head
#   stress tools/dbg/head_stress.py: repeatability of the head and the split path (raw and with BN)
#   trace  rocprofv3 kernel stats of one step kind each (TRACES="mode batch views;..."): cfg-2 eval, cfg-2
#          train-mode BN (test.py:61), cfg-3 eval; per step = over 3 warm-up + 5 timed steps
# Every GPU step has its own time limit; the script stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; TAG=${1:-r6}; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
STAGES=${*:-tests smoke bench prof pmc}
has() { case " $STAGES " in *" $1 "*) return 0;; esac; return 1; }
if has tests; then
  MVS_PARITY_OUT=$OUT/parity timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rf --timeout 600 \
    --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20; tail -2 $OUT/pytest_gpu.log
  if [ $rc -gt 1 ]; then exit $rc; fi
fi
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
fi
if has bench; then
  s=$(date +%s); timeout -k 10 900 python bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err; rc=$?
  echo "bench rc=$rc wall=$(( $(date +%s) - s ))s"
  if [ $rc -ne 0 ]; then tail -20 $OUT/bench.err; exit $rc; fi
  python3 - $OUT/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("value %.1f maps/s, %.3f ms/step; head %s" % (d["value"], d["ms_per_step"], {k: r.get(k) for k in ("kernel_ms", "achieved", "frac", "traffic")}))
for k in ("exact_fp32_step", "train_bn", "train_step", "cost_volume_backward", "e2e_configs", "kernel_configs"):
    if k in d:
        print(k, json.dumps(d[k])[:400])
PY
fi
if has prof; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra --no-train-step > $OUT/prof_bench.json 2> $OUT/prof_bench.err
  rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
  f=$(ls $OUT/prof/*/run_kernel_stats.csv $OUT/prof/run_kernel_stats.csv 2>/dev/null | head -1); head -14 "$f" | cut -c1-160
fi
if has cfgprof; then   # per-config warp-kernel stats (bench kernel_configs legs: cfg 3/5 channel quads, cfg 4 NCDHW)
  for c in 2 3 4 5; do
    q=1; [ $c = 4 ] && q=0
    MVS_BENCH_C4=$q timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/cfg$c" \
      -o cfg$c -- python3 tools/kernel_bench.py $c > $OUT/cfg$c.log 2>&1; rc=$?
    echo "cfgprof $c rc=$rc"; grep '^{' $OUT/cfg$c.log; [ $rc -ne 0 ] && exit $rc
  done
fi
if has evalprof; then   # the value leg alone: fp32 cfg-2 eval steps (tools/eval_steps.py)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/eval" -o eval -- \
    python3 tools/eval_steps.py --steps 10 > $OUT/evalprof.log 2>&1; rc=$?; echo "evalprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
if has pmc; then
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" \
      "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES" \
      "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
      "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp -d "$GRAFT_REPO_ROOT/$OUT/hpmc/p$i" -o run --output-format csv -- \
      python3 tools/hip_reg_layers.py --only ${PMC_LAYER:-cv_head} --reps 3 > $OUT/hpmc_p$i.log 2>&1
    rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/hpmc_p$i.log; exit $rc; }
  done
  python3 tools/summarize_pmc.py $OUT/hpmc ${PMC_KERNEL:-cv_head_kernel} > $OUT/head_pmc.json; cat $OUT/head_pmc.json
fi
if has stress; then
  timeout -k 10 400 python -u tools/dbg/head_stress.py ${STRESS_N:-40} > $OUT/head_stress.log 2>&1; rc=$?
  echo "stress rc=$rc"; grep -E "cfg|differs" $OUT/head_stress.log | head -40; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 400 python -u tools/dbg/head_stress.py ${STRESS_N:-40} bn > $OUT/head_stress_bn.log 2>&1; rc=$?
  echo "stress bn rc=$rc"; grep -E "cfg|differs" $OUT/head_stress_bn.log | head -40; [ $rc -ne 0 ] && exit $rc
fi
if has trace; then
  IFS=';' read -ra TRACES <<< "${TRACES:-eval 4 3 fp32;train 4 3 fp32;eval 8 5 fp32}"
  for m in "${TRACES[@]}"; do set -- $m; a=${4:-fp32}; t=tr_$1_v$3_$a
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/$t" -o run --output-format csv -- \
      python3 tools/step_trace.py --mode $1 --batch $2 --views $3 --arithmetic $a --steps 5 > $OUT/$t.log 2>&1
    rc=$?; echo "trace $t rc=$rc"; grep "step" $OUT/$t.log | tail -2; [ $rc -ne 0 ] && exit $rc
    f=$(ls $OUT/$t/*/run_kernel_stats.csv $OUT/$t/run_kernel_stats.csv 2>/dev/null | head -1)
    python3 tools/kstats.py "$f" 8 24
  done
fi
exit 0
