#!/bin/bash
# 2-D encoder convs: per-layer time and output checksums, shipped library and tools/exp_libs variants
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-enc}; mkdir -p $OUT; export TMPDIR=/tmp
for v in default ${VARIANTS:-c2old}; do
  if [ $v != default ]; then L=$GRAFT_REPO_ROOT/tools/exp_libs/lib$v.so; else L=; fi
  echo "== $v"; MVS_LIB_PATH=$L timeout -k 10 240 python -u tools/enc_layers.py --reps 20 > $OUT/$v.log 2>&1 || { tail -20 $OUT/$v.log; exit 1; }
  cat $OUT/$v.log
done
