# GPU: parity tests of the fused path (TESTS, default the parity file), then library variants.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -m gpu -x -v -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | tail -6
if [ $rc -ne 0 ]; then exit $rc; fi
VARIANTS="${VARIANTS:-base:}" CFGS="${CFGS:-2 3}" bash tools/exp_variants.sh
