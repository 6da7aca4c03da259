# GPU round check: parity tests, kernel timings, rocprof kernel stats.  Run from the repo root.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/kernel_bench.py > gpurun_out/kernel_bench.log 2>&1; rc=$?; echo "kbench rc=$rc"; cat gpurun_out/kernel_bench.log | grep -v amdgpu.ids
if [ $rc -ne 0 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/kernel_bench.py" 2 > gpurun_out/prof.log 2>&1; echo "prof rc=$?"
cat gpurun_out/prof/run_kernel_stats.csv | cut -c1-250
