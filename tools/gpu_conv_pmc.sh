# PMC passes over tools/conv_bench.py with library variant $1 (tools/exp_libs/lib$1.so)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
export MVS_LIB_PATH="$GRAFT_REPO_ROOT/tools/exp_libs/lib$1.so"
timeout -k 10 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$1_a" -o run --output-format csv -- python3 tools/conv_bench.py 5 || exit $?
timeout -k 10 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$1_b" -o run --output-format csv -- python3 tools/conv_bench.py 5 || exit $?
timeout -k 10 90 rocprofv3 --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_ICACHE_MISSES GRBM_GUI_ACTIVE -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$1_c" -o run --output-format csv -- python3 tools/conv_bench.py 5 || exit $?
