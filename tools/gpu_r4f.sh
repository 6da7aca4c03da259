#!/bin/bash
# round 4: head race check (300 cfg-2 launches against the split path), head timing, new parity tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-r4f}; mkdir -p $OUT; export TMPDIR=/tmp
HEAD_DIFF_BIG=300 HEAD_DIFF_QUIET=1 HEAD_DIFF_FULLBOX=1 timeout -k 10 300 python -u tools/dbg/head_diff.py > $OUT/race.log 2>&1 || exit 1
grep -E "^runs|y0 bad [0-9]" $OUT/race.log | head -20
timeout -k 10 200 python -u tools/hip_reg_layers.py --only cv_head,cv_split --reps 10 2>&1 | grep -E "^cv_" || exit 1
MVS_PARITY_OUT=$OUT/parity timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_cv_head.py \
  "tests/test_split_conv.py::test_split_conv_dynamic_range" \
  "tests/test_gpu_configs.py::test_cfg2_depth_flips_within_reference_self_noise" \
  "tests/test_gpu_configs.py::test_model_end_to_end_at_cfg3_cfg5" > $OUT/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|passed|failed|^PARITY" $OUT/pytest.log | cut -c1-400 | tail -30
exit $rc
