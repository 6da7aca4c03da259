# fused forward kernel: timings (NCDHW / channel-quad) and PMC passes at cfg2 (channel-quad)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
[ -n "$1" ] && export MVS_LIB_PATH="$GRAFT_REPO_ROOT/tools/exp_libs/lib$1.so"
timeout -k 10 120 python3 -u tools/kernel_bench.py 2 3 4 5 || exit $?
MVS_BENCH_C4=1 timeout -k 10 120 python3 -u tools/kernel_bench.py 2 3 5 || exit $?
export MVS_BENCH_C4=1
PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE;GRBM_GUI_ACTIVE GRBM_COUNT" bash tools/pmc_prog.sh fwd_pmc${1} tools/kernel_bench.py 2
