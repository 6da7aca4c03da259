#!/bin/bash
# Round 3: the new train / end-to-end tests, one pytest per file (failure details printed per file).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r3d
mkdir -p $OUT
export MVS_PARITY_OUT=$OUT/parity
fail=0
for f in tests/test_gpu_train.py tests/test_gpu_configs.py; do
  n=$(basename $f .py)
  timeout -k 10 600 python -u -m pytest $f -m gpu -v -s --tb=short --timeout 500 --timeout-method thread \
      > $OUT/$n.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|PARITY|Error|^E |^\[|train step" $OUT/$n.log | cut -c1-500 | head -60
  if [ $rc -gt 1 ]; then echo "$f rc=$rc: stopping"; exit $rc; fi
  [ $rc -ne 0 ] && fail=1
done
exit $fail
