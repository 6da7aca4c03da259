#!/bin/bash
# Round 3: split-fp16 conv_0_0 -- its parity tests, the train-step / e2e tests, per-layer times, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r3h
mkdir -p $OUT
export TMPDIR=/tmp MVS_PARITY_OUT=$OUT/parity
timeout -k 10 300 python -u -m pytest tests/test_split_conv.py tests/test_gpu_train.py tests/test_gpu_configs.py -m gpu -v -s \
    --timeout 250 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|split |^E " $OUT/pytest.log | cut -c1-300 | head -60; tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 python -u tools/hip_reg_layers.py > $OUT/reg_layers.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/reg_layers.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"; tail -3 $OUT/bench.err
exit $rc
