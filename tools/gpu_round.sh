# Full GPU round: parity tests, kernel timings, bench (+CPU baseline), rocprof stats, PMC traffic.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
fi
timeout -k 10 300 python tools/kernel_bench.py > gpurun_out/kernel_bench.log 2>&1; rc=$?; echo "kbench rc=$rc"; grep cfg gpurun_out/kernel_bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
s=$(date +%s); timeout -k 10 900 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err; rc=$?; echo "bench rc=$rc wall=$(( $(date +%s) - s ))s"; tail -1 gpurun_out/bench.log | cut -c1-200
mkdir -p gpurun_out/miopen_db && cp -r tools/miopen_db/. gpurun_out/miopen_db/ 2>/dev/null
if [ $rc -ne 0 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/kernel_bench.py" 2 > gpurun_out/prof.log 2>&1; echo "prof rc=$?"
head -6 gpurun_out/prof/run_kernel_stats.csv | cut -c1-160
bash tools/pmc.sh pmc 2
