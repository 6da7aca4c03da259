# PMC passes (one counter group per pass, kernel-trace only) over an arbitrary python program.
# Usage (on the GPU box, repo root): bash tools/pmc_prog.sh <outdir> <script.py> [args...]
# PMC_GROUPS (optional, ';'-separated) overrides the default counter groups.
OUT="$GRAFT_REPO_ROOT/gpurun_out/$1"; shift; mkdir -p "$OUT"
export TMPDIR=/tmp
DEFAULT="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE"
IFS=';' read -ra GROUPS_ <<< "${PMC_GROUPS:-$DEFAULT}"
i=0
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- python3 "$@" > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
exit 0
