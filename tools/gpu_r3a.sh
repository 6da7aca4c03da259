#!/bin/bash
# Round 3, first GPU pass: full -m gpu suite (parity numbers recorded), then the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r3a
mkdir -p $OUT
export MVS_PARITY_OUT=$OUT/parity
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --maxfail=5 --timeout 300 --timeout-method thread \
    > $OUT/pytest.log 2>&1
rc=$?
tail -5 $OUT/pytest.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
brc=$?
tail -3 $OUT/bench.err
exit $brc
