#!/bin/bash
# round 5: bound-word update variants (main: slot read before the atomic at kernel ends; nochk: always
# the atomic) -- eval / train-mode step times (tools/step_trace.py, 20 steps) and the head alone
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-r5bab}; shift; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
for v in ${*:-main nochk}; do
  if [ "$v" = main ]; then unset MVS_LIB_PATH; else export MVS_LIB_PATH=$GRAFT_REPO_ROOT/tools/exp_libs/lib$v.so; fi
  timeout -k 10 200 python -u tools/step_trace.py --mode eval --steps 20 > $OUT/${v}_eval$rep.log 2>&1 || exit 1
  timeout -k 10 200 python -u tools/step_trace.py --mode train --steps 10 > $OUT/${v}_train$rep.log 2>&1 || exit 1
  echo "== $v: $(grep step $OUT/${v}_eval$rep.log | tail -1)  $(grep step $OUT/${v}_train$rep.log | tail -1)"
done
done
