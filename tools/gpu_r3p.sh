#!/bin/bash
# PMC passes over one layer of tools/hip_reg_layers.py: bash tools/gpu_r3p.sh <tag> <layer> <kernel-substring>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=$1; L=$2; K=$3
export TMPDIR=/tmp
PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY;SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES;FETCH_SIZE;WRITE_SIZE" \
  bash tools/pmc_prog.sh $T tools/hip_reg_layers.py --only $L --reps 5 || exit $?
python3 tools/summarize_pmc.py gpurun_out/$T $K
