#!/bin/bash
# quick check: the GPU tests matching $K, then the eval-step time (and $LAYERS per layer)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-quick}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "$K" > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $OUT/pytest.log | head; exit $rc; }
timeout -k 10 240 python -u tools/hip_reg_layers.py --only ${LAYERS:-step} --reps 20 2>&1 | grep -E "ms$"
