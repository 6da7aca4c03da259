# Round bench: the driver's default bench line, then rocprofv3 kernel stats of the same command
# (CPU baseline skipped under the profiler) -- usage: bash tools/gpu_bench_round.sh <tag>
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r02}
timeout -k 10 600 python3 -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err; rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/${T}_bench.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${T}_prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/${T}_prof_bench.json 2> gpurun_out/${T}_prof_bench.err; rc=$?; echo "prof rc=$rc"
exit $rc
