#!/bin/bash
# split-head timing ablations: tools/dbg/head_time.py under library variants (tools/exp_libs/lib<v>.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-ptime}; shift; mkdir -p $OUT; export TMPDIR=/tmp
for v in ${*:-main pA pM pC}; do
  if [ "$v" = main ]; then unset MVS_LIB_PATH; else export MVS_LIB_PATH=$GRAFT_REPO_ROOT/tools/exp_libs/lib$v.so; fi
  timeout -k 10 200 python -u tools/dbg/head_time.py 20 > $OUT/$v.log 2>&1; rc=$?
  echo "== $v rc=$rc"; grep -E "^cfg" $OUT/$v.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
