# PMC HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the roofline kernel (channel-quad
# fused forward, cfg 2) and of the backward (cfg 2, + instruction mix), kernel-trace only
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
MVS_BENCH_C4=1 PMC_GROUPS="FETCH_SIZE;WRITE_SIZE" bash tools/pmc_prog.sh fwd_traffic tools/kernel_bench.py 2 || exit $?
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE" bash tools/pmc_prog.sh bwd_pmc_final tools/bwd_bench.py 2
