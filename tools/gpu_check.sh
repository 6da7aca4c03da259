cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --kernel-only --no-cpu-baseline --kernel-iters 20 > gpurun_out/bench_kernel.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench_kernel.log
if [ $rc -ne 0 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof1" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --kernel-only --no-cpu-baseline --kernel-iters 10 > gpurun_out/prof1.log 2>&1; echo "prof rc=$?"
ls -R gpurun_out/prof1 | head
