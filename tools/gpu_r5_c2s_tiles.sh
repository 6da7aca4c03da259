#!/bin/bash
# round 5: conv2d_split tile shapes (MVS_C2S_TILE 0 / 1 / 2): parity tests and per-layer times for each
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-r5c2s}; mkdir -p $OUT; export TMPDIR=/tmp
for t in 0 1 2; do
  MVS_C2S_TILE=$t timeout -k 10 300 python -u -m pytest tests/test_conv2d_split.py -m gpu -q -x --timeout 120 \
    --timeout-method thread > $OUT/pytest_t$t.log 2>&1 || { echo "tile $t tests failed"; tail -30 $OUT/pytest_t$t.log; exit 1; }
  MVS_C2S_TILE=$t timeout -k 10 300 python -u tools/enc_layers.py > $OUT/enc_t$t.log 2>&1 || { tail $OUT/enc_t$t.log; exit 1; }
  echo "== tile $t: $(tail -1 $OUT/pytest_t$t.log)"; grep -E "^conv2d|split16 raising|per eval|feature_encoder" $OUT/enc_t$t.log | grep -v "1  sha\|32  sha" 
done
