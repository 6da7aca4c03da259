#!/bin/bash
# Round 3: the new end-to-end / train tests with progress lines (find-db as committed).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r3d
mkdir -p $OUT
timeout -k 10 240 python -u tools/hip_reg_layers.py > $OUT/reg_layers.log 2>&1
cat $OUT/reg_layers.log | grep -v amdgpu.ids
export MVS_PARITY_OUT=$OUT/parity
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_train.py -m gpu -v -s \
    --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|PARITY|Error|^E |^\[|train step" $OUT/pytest.log | cut -c1-600 | head -80
exit $rc
