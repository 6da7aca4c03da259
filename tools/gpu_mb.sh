cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -w -o /tmp/atomic_patterns tools/microbench/atomic_patterns.hip || exit 1
timeout -k 10 120 /tmp/atomic_patterns > gpurun_out/atomic_patterns3.log 2>&1; rc=$?; cat gpurun_out/atomic_patterns3.log; exit $rc
