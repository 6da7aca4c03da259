# Round 2: backward PMC counters, atomics microbench v2, cfg-2 e2e parity test
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -w -o /tmp/atomic_patterns tools/microbench/atomic_patterns.hip || exit 1
timeout -k 10 120 /tmp/atomic_patterns > gpurun_out/atomic_patterns2.log 2>&1; rc=$?; cat gpurun_out/atomic_patterns2.log; [ $rc -ne 0 ] && exit $rc
bash tools/pmc_prog.sh r2d_bwd_pmc tools/bwd_bench.py 2 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -rf --timeout 300 --timeout-method thread -k "cfg2" > gpurun_out/r2d_pytest_cfg2.log 2>&1; rc=$?; echo "pytest cfg2 rc=$rc"; tail -15 gpurun_out/r2d_pytest_cfg2.log
exit $rc
