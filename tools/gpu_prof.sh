# rocprofv3 kernel-trace stats of the fused op at one config (default cfg 2) -> gpurun_out/prof_<tag>/
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-cur}; CFG=${CFG:-2}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/kernel_bench.py" $CFG > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; cut -d, -f1-4 gpurun_out/prof_$TAG/run_kernel_stats.csv | cut -c1-150
exit $rc
