cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
VARIANTS="base: pg2:-DMVS_EXP_PG=2 pg8:-DMVS_EXP_PG=8" CFGS="2 3 4 5" bash tools/exp_variants.sh
