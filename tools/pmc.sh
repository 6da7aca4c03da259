# PMC passes (one counter group per pass, kernel-trace only) on the fused kernel of one config.
# Usage (on the GPU box, repo root): bash tools/pmc.sh <outdir> [cfg]
# PMC_GROUPS (optional, ';'-separated) overrides the default counter groups.
OUT="$GRAFT_REPO_ROOT/gpurun_out/${1:-pmc}"; CFG="${2:-2}"; mkdir -p "$OUT"
export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
DEFAULT="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE;TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
IFS=';' read -ra GROUPS_ <<< "${PMC_GROUPS:-$DEFAULT}"
i=0
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/kernel_bench.py" $CFG > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
exit 0
