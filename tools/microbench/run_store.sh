cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o /tmp/store_patterns tools/microbench/store_patterns.hip || exit 1
timeout -k 10 120 /tmp/store_patterns | tee gpurun_out/store_patterns.log
