#!/bin/bash
# head race experiment: repeatability of cv_head under library variants (tools/exp_libs/lib<v>.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-hexp}; shift; mkdir -p $OUT; export TMPDIR=/tmp
for v in ${*:-v0 vA vC vN}; do
  MVS_LIB_PATH=$GRAFT_REPO_ROOT/tools/exp_libs/lib$v.so HEAD_STRESS_CFGS="${CFGS:-1,2,20,24,40;1,3,16,29,41}" \
    timeout -k 10 300 python -u tools/dbg/head_stress.py ${N:-60} > $OUT/$v.log 2>&1; rc=$?
  echo "== $v rc=$rc"; grep -E "^cfg" $OUT/$v.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
