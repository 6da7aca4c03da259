cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
/opt/rocm/bin/hipcc -O3 -w --offload-arch=gfx950 -o /tmp/gather_patterns tools/microbench/gather_patterns.hip || exit 1
timeout -k 10 120 /tmp/gather_patterns | tee gpurun_out/gather_patterns.log
