#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/dbg; export TMPDIR=/tmp
for v in ${VARIANTS:-default default}; do
  echo "== $v"
  if [ $v != default ]; then export MVS_LIB_PATH=$GRAFT_REPO_ROOT/tools/exp_libs/lib$v.so; else unset MVS_LIB_PATH; fi
  timeout -k 10 200 python -u tools/dbg/head_diff.py 2>&1 | grep -v amdgpu.ids || exit 1
done
