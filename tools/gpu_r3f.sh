#!/bin/bash
# Round 3: MIOpen find for the cfg-5 live-region torch reference (the cfg-5 e2e test's reference path).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r3f
mkdir -p $OUT gpurun_out/miopen_db
cp tools/miopen_db/*.txt gpurun_out/miopen_db/ 2>/dev/null
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
timeout -k 10 900 python -u tools/miopen_find.py cfg5_live_torch > $OUT/find.log 2>&1
rc=$?
grep -v "^\.\.\.\|\[bench" $OUT/find.log | tail -8
exit $rc
