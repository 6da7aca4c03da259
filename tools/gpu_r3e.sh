#!/bin/bash
# Round 3: region-conv kernel changes -- parity subset, per-layer alone times and the eval step on
# 3 / 2 / 1 streams, PMC of S2 conv_1_0 alone.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r3e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_bf16_cost_volume.py -m gpu -q -x \
    -k "region or live or channel_quad or bf16 or mvsnet or narrow" --timeout 200 --timeout-method thread \
    > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" $OUT/pytest.log | head -20; exit $rc; fi
timeout -k 10 240 python -u tools/hip_reg_layers.py > $OUT/reg_layers.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/reg_layers.log
if [ $rc -ne 0 ]; then exit $rc; fi
PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY;SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F32 SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE;TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum;FETCH_SIZE" \
  bash tools/pmc_prog.sh r3e/pmc_conv_1_0 tools/hip_reg_layers.py --only conv_1_0 --reps 5
rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY;SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
  bash tools/pmc_prog.sh r3e/pmc_conv_0_0 tools/hip_reg_layers.py --only conv_0_0 --reps 5
