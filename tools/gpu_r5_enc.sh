#!/bin/bash
# round 5: split-fp16 encoder convolutions -- GPU tests of the new kernel, per-layer times, encoder totals
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-r5enc}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_conv2d_split.py -m gpu -v -rf --timeout 120 --timeout-method thread \
  > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -15
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/enc_layers.py > $OUT/enc.log 2>&1 && \
MVS_CONV2D_F16=0 timeout -k 10 300 python -u tools/enc_layers.py --reps 5 2>&1 | tail -1 >> $OUT/enc.log; rc=$?
cat $OUT/enc.log; exit $rc
