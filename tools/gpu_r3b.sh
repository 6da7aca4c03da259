#!/bin/bash
# Round 3: MIOpen find-db for the full-volume reference leg and the train step at every BASELINE
# config (so no test or bench falls back to MIOpen's naive 3-D kernels), then the new end-to-end tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r3b
mkdir -p $OUT gpurun_out/miopen_db
cp tools/miopen_db/*.txt gpurun_out/miopen_db/ 2>/dev/null
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -w -o /tmp/store_c4 tools/microbench/store_c4_patterns.hip && \
    timeout -k 10 120 /tmp/store_c4 > $OUT/store_c4_patterns.log 2>&1
cat $OUT/store_c4_patterns.log
timeout -k 10 780 python -u tools/miopen_find.py > $OUT/find.log 2>&1
rc=$?
tail -12 $OUT/find.log
if [ $rc -ne 0 ]; then echo "find rc=$rc"; exit $rc; fi
export MVS_PARITY_OUT=$OUT/parity
timeout -k 10 360 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_train.py -m gpu -v -s \
    --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|PARITY|Error|^E " $OUT/pytest.log | head -60
exit $rc
