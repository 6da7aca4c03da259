#!/bin/bash
# Round 3 baseline: full GPU suite (durations), smoke, the driver's bench line, rocprof kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-r03g}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp MVS_PARITY_OUT=$OUT/parity
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --durations=25 --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -35 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_bench_round.sh $T
