#!/bin/bash
# round 5: train-mode BN path -- its parity tests (region split sums, live == full volume, end to end) and
# a per-kernel trace of the train-mode step
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-r5tr}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_region_split.py tests/test_bn_train_params.py tests/test_gpu_parity.py tests/test_gpu_train.py \
  -m gpu -v -rf --timeout 300 --timeout-method thread -k "sums_and_store_box or train_mode or end_to_end or region_split or bn_train or encoder" \
  > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -15
[ $rc -ne 0 ] && exit $rc
TRACES="train 4 3" bash tools/gpu_r5.sh ${1:-r5tr} trace
