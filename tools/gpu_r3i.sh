#!/bin/bash
# Round 3: the whole GPU suite after the split-fp16 conv_0_0 became the eval default, per-layer times, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r3i
mkdir -p $OUT
export TMPDIR=/tmp MVS_PARITY_OUT=$OUT/parity
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --durations=12 --timeout 250 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "FAILED|^E |passed|failed" $OUT/pytest.log | cut -c1-300 | head -40; tail -16 $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 python -u tools/hip_reg_layers.py > $OUT/reg_layers.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/reg_layers.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"; tail -3 $OUT/bench.err
exit $rc
