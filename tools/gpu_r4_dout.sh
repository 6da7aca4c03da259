#!/bin/bash
# fused deconv_1_0 + conv_out: bit-equality tests, then the eval step with / without it
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-r4d}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_gpu_parity.py::test_deconv_out_equals_deconv_then_conv_out" tests/test_cv_head.py::test_mvsnet_head_equals_split_volume_path \
  > $OUT/pytest.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|passed|failed" $OUT/pytest.log | tail -12
if [ $rc -ne 0 ]; then exit $rc; fi
for v in 1 0; do
  MVS_DECONV_OUT=$v timeout -k 10 300 python -u tools/step_trace.py --mode eval 2>&1 | grep "step:" | sed "s/^/deconv_out=$v /"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/eval" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/step_trace.py" --mode eval > $OUT/eval.log 2>&1; echo "prof rc=$?"
grep -E "deconv_out|deconv3d|narrow_kernel<1|cv_head" $OUT/eval/run_kernel_stats.csv | cut -c1-160
