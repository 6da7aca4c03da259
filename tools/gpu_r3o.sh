#!/bin/bash
# Round 3: the stride-2 split conv_1_0 -- its tests, per-layer times, the eval-path parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r3o}
mkdir -p $OUT
export TMPDIR=/tmp MVS_PARITY_OUT=$OUT/parity
timeout -k 10 200 python -u -m pytest tests/test_split_conv.py -m gpu -q -s --timeout 100 --timeout-method thread > $OUT/split_tests.log 2>&1
rc=$?; grep -E "split |s2 |passed|failed|Error" $OUT/split_tests.log | head -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u tools/hip_reg_layers.py > $OUT/reg_layers.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/reg_layers.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -q -k "end_to_end or channel_quad or live or sharded" --timeout 250 --timeout-method thread > $OUT/e2e.log 2>&1
rc=$?; grep -E "passed|failed|^E |FAILED" $OUT/e2e.log | head -20
exit $rc
