cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/kernel_bench.py > gpurun_out/kernel_bench.log 2>&1; rc=$?; echo "kbench rc=$rc"; grep cfg gpurun_out/kernel_bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
s=$(date +%s); timeout -k 10 900 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_search.log 2>&1; rc=$?; echo "bench(search on) rc=$rc wall=$(( $(date +%s) - s ))s"; tail -1 gpurun_out/bench_search.log | cut -c1-300
