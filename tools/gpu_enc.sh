#!/bin/bash
# 2-D encoder convs: per-layer time and output checksums under each MVS_CONV2D_SPLIT value in $SPLITS
# ("auto" = the launcher's choice)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-enc}; mkdir -p $OUT; export TMPDIR=/tmp
for v in ${SPLITS:-auto 1}; do
  if [ $v != auto ]; then export MVS_CONV2D_SPLIT=$v; else unset MVS_CONV2D_SPLIT; fi
  echo "== split $v"; timeout -k 10 240 python -u tools/enc_layers.py --reps 20 > $OUT/s$v.log 2>&1 || { tail -20 $OUT/s$v.log; exit 1; }
  grep -v amdgpu.ids $OUT/s$v.log
done
