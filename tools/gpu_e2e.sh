# GPU tests, then the bench (with its full-volume regulariser comparison), then a kernel-trace
# profile of a short bench run (where the end-to-end step time goes).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
fi
s=$(date +%s); timeout -k 10 900 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err; rc=$?; echo "bench rc=$rc wall=$(( $(date +%s) - s ))s"; tail -1 gpurun_out/bench.log | cut -c1-400
if [ $rc -ne 0 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_e2e" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --kernel-iters 5 > gpurun_out/prof_e2e.log 2>&1; echo "prof rc=$?"
head -12 gpurun_out/prof_e2e/run_kernel_stats.csv | cut -c1-180
