# Kernel experiments on the GPU box: optional GPU parity tests, then variants of the library built with
# -D flags (tools/exp_variants.sh), then optionally the store-pattern microbenchmark.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
VARIANTS="${VARIANTS:-base:}" CFGS="${CFGS:-2 3}" bash tools/exp_variants.sh || exit $?
if [ -n "$STORE_MB" ]; then bash tools/microbench/run_store.sh; fi
