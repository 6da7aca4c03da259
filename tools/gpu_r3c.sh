#!/bin/bash
# Round 3: remaining MIOpen find shapes (cfg 5 full volume, the train-step test shapes), then the new
# end-to-end / train tests with progress lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r3c
mkdir -p $OUT gpurun_out/miopen_db
cp tools/miopen_db/*.txt gpurun_out/miopen_db/ 2>/dev/null
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
timeout -k 10 600 python -u tools/miopen_find.py cfg5_full cfg1_train smooth_train > $OUT/find.log 2>&1
rc=$?
grep -v "^\.\.\.\|\[bench" $OUT/find.log | tail -8
if [ $rc -ne 0 ]; then echo "find rc=$rc"; exit $rc; fi
export MVS_PARITY_OUT=$OUT/parity
timeout -k 10 420 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_train.py -m gpu -v -s \
    --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|PARITY|Error|^E |^\[" $OUT/pytest.log | cut -c1-400 | head -60
exit $rc
