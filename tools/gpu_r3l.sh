#!/bin/bash
# Round 3: rocprof kernel stats of the bench command and PMC passes over the split conv_0_0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-r3l}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof_bench.err; rc=$?; echo "prof rc=$rc"
[ $rc -ne 0 ] && exit $rc
head -25 $OUT/prof/run_kernel_stats.csv | cut -d, -f1-6 | cut -c1-200
PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY;SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES;FETCH_SIZE;WRITE_SIZE" \
  bash tools/pmc_prog.sh $T/pmc_split tools/hip_reg_layers.py --only conv_0_0_split --reps 5
rc=$?; [ $rc -ne 0 ] && exit $rc
python3 tools/summarize_pmc.py $OUT/pmc_split conv0_split_kernel
