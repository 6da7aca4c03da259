#!/bin/bash
# Round 3: split conv_0_0 tests + per-layer times, bench (default line), rocprof kernel stats of the same
# command, PMC of the split conv_0_0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r3j}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_split_conv.py -m gpu -q -s --timeout 100 --timeout-method thread > $OUT/split_tests.log 2>&1
rc=$?; grep -E "split |passed|failed" $OUT/split_tests.log | head -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u tools/hip_reg_layers.py > $OUT/reg_layers.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/reg_layers.log; [ $rc -ne 0 ] && exit $rc
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 500 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"; tail -4 $OUT/bench.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof_bench.err; rc=$?; echo "prof rc=$rc"
[ $rc -ne 0 ] && exit $rc
PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY;SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES;FETCH_SIZE;WRITE_SIZE" \
  bash tools/pmc_prog.sh ${1:-r3j}/pmc_split tools/hip_reg_layers.py --only conv_0_0_split --reps 5
