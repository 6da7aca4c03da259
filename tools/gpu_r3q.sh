#!/bin/bash
# Round 3: split cost volume -- split tests, per-layer times, e2e/model tests, bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r3q}
mkdir -p $OUT
export TMPDIR=/tmp MVS_PARITY_OUT=$OUT/parity
timeout -k 10 200 python -u -m pytest tests/test_split_conv.py -m gpu -q -s --timeout 100 --timeout-method thread > $OUT/split_tests.log 2>&1
rc=$?; grep -E "passed|failed|Error|^E " $OUT/split_tests.log | head -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u tools/hip_reg_layers.py > $OUT/reg_layers.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/reg_layers.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -q -k "end_to_end or channel_quad or live or sharded" --timeout 250 --timeout-method thread > $OUT/e2e.log 2>&1
rc=$?; grep -E "passed|failed|^E |FAILED" $OUT/e2e.log | head -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-extra > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"; grep "bench " $OUT/bench.err | tail -8
exit $rc
