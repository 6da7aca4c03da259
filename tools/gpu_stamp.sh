#!/bin/bash
# cv_head segment stamps at cfg 2 (diagnostic build tools/exp_libs/libstamp.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-stamp}; mkdir -p $OUT; export TMPDIR=/tmp
rm -f $OUT/stamps.bin
MVS_LIB_PATH=$GRAFT_REPO_ROOT/tools/exp_libs/libstamp.so MVS_HEAD_STAMPS=$OUT/stamps.bin timeout -k 10 200 \
  python -u tools/hip_reg_layers.py --only cv_head --reps 2 2>&1 | grep -E "^cv_" || exit 1
python3 tools/dbg/stamps.py $OUT/stamps.bin
rm -f $OUT/stamps.bin
