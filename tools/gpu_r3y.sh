#!/bin/bash
# store-pattern microbenchmark of the channel-quad volume, PMC traffic of the split-store fused kernel,
# per-layer times (packed split conversion)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r3y; export TMPDIR=/tmp
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o /tmp/store_c4 tools/microbench/store_c4_patterns.hip || exit 1
timeout -k 10 120 /tmp/store_c4 > gpurun_out/r3y/store_c4.log 2>&1; rc=$?; cat gpurun_out/r3y/store_c4.log; [ $rc -ne 0 ] && exit $rc
MVS_BENCH_C4=1 PMC_GROUPS="FETCH_SIZE;WRITE_SIZE" bash tools/pmc_prog.sh r3y/fwd_traffic tools/kernel_bench.py 2 || exit $?
python3 tools/summarize_pmc.py gpurun_out/r3y/fwd_traffic "cost_volume_staged_kernel<3, 8, 32>"
timeout -k 10 240 python -u tools/hip_reg_layers.py > gpurun_out/r3y/reg_layers.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r3y/reg_layers.log
exit $rc
