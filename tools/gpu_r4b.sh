#!/bin/bash
# Round 4: fused head (cv_head.hip) parity against the split path, then per-layer / step times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r4b}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_cv_head.py -m gpu -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|^E " $OUT/pytest.log | cut -c1-300 | head -40; tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/hip_reg_layers.py > $OUT/reg_layers.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/reg_layers.log
exit $rc
