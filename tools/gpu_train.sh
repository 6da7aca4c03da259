#!/bin/bash
# training path: GPU train tests, then the cfg-2 train step alone under a rocprofv3 kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-train}; mkdir -p $OUT; export TMPDIR=/tmp
MVS_PARITY_OUT=$OUT/parity timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_train.py \
  > $OUT/pytest.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|passed|failed" $OUT/pytest.log | cut -c1-300 | tail -20
[ $rc -ne 0 ] && exit $rc
MVS_TRAIN_MARK=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/proft" -o run --output-format csv -- \
  python3 tools/train_step_prof.py > $OUT/prof_train.log 2>&1; echo "train prof rc=$?"; grep ms_per_step $OUT/prof_train.log
python3 tools/trace_between_marks.py $(ls $OUT/proft/*/run_kernel_trace.csv $OUT/proft/run_kernel_trace.csv 2>/dev/null | head -1) 15 | tee $OUT/train_step_kernels.txt
timeout -k 10 300 python3 tools/train_step_prof.py > $OUT/train.log 2>&1; echo "train rc=$?"; grep ms_per_step $OUT/train.log
