cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/r6x; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -v --timeout 600 --timeout-method thread -k "fp32_head or cfg3_cfg5 or flips" > $OUT/pytest.log 2>&1; rc=$?
echo "rc=$rc"; grep -E "PASSED|FAILED|^E " $OUT/pytest.log | head -30; exit $rc
