# GPU round check: parity tests, kernel timings, e2e bench, rocprof kernel stats.  Repo root.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/kernel_bench.py > gpurun_out/kernel_bench.log 2>&1; rc=$?; echo "kbench rc=$rc"; grep cfg gpurun_out/kernel_bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 5 --warmup 2} > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_bench" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1; echo "prof rc=$?"
head -12 gpurun_out/prof_bench/run_kernel_stats.csv | cut -c1-200
