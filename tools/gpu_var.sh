#!/bin/bash
# time named layers of the eval step (tools/hip_reg_layers.py --only $LAYERS) for the shipped library
# and each tools/exp_libs variant in $VARIANTS
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-var}; mkdir -p $OUT; export TMPDIR=/tmp
for v in default $VARIANTS; do
  if [ $v != default ]; then L=$GRAFT_REPO_ROOT/tools/exp_libs/lib$v.so; else L=; fi
  echo "== $v"; MVS_LIB_PATH=$L timeout -k 10 240 python -u tools/hip_reg_layers.py --only ${LAYERS:-step} --reps ${REPS:-20} > $OUT/$v.log 2>&1 || { tail -20 $OUT/$v.log; exit 1; }
  grep -E "ms$" $OUT/$v.log
done
