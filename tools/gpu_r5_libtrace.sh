#!/bin/bash
# per-kernel step traces under library variants: bash tools/gpu_r5_libtrace.sh <tag> <mode> <batch> <views> <lib>...
# (lib "main" = the in-tree build; else tools/exp_libs/lib<v>.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/$1; MODE=$2; BATCH=$3; VIEWS=$4; shift 4; mkdir -p $OUT; export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = main ]; then unset MVS_LIB_PATH; else export MVS_LIB_PATH=$GRAFT_REPO_ROOT/tools/exp_libs/lib$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/$v" -o run --output-format csv -- \
    python3 tools/step_trace.py --mode $MODE --batch $BATCH --views $VIEWS --steps 5 > $OUT/$v.log 2>&1
  rc=$?; echo "== $v rc=$rc $(grep step $OUT/$v.log | tail -1)"; [ $rc -ne 0 ] && exit $rc
  f=$(ls $OUT/$v/*/run_kernel_stats.csv $OUT/$v/run_kernel_stats.csv 2>/dev/null | head -1)
  python3 tools/kstats.py "$f" 8 40 | grep -E "region|kernel time"
done
exit 0
