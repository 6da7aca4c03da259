#!/bin/bash
# Round 3: split conv_0_0 tests + per-layer times, train-step tests with the tap-GEMM training convs,
# the default bench line and the opt-in train-step field.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r3k}
mkdir -p $OUT
export TMPDIR=/tmp MVS_PARITY_OUT=$OUT/parity
NO_BENCH=1 bash tools/gpu_r3j.sh ${1:-r3k} || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -m gpu -v -s --durations=5 --timeout 300 --timeout-method thread > $OUT/train_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|^E |s call" $OUT/train_tests.log | cut -c1-250 | head -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"; grep "bench " $OUT/bench.err | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-extra --train-step > $OUT/bench_train.json 2> $OUT/bench_train.err; rc=$?; echo "bench train rc=$rc"; tail -3 $OUT/bench_train.err
exit $rc
