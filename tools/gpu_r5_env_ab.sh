#!/bin/bash
# round 5: A/B of an environment switch on the eval step (tools/step_trace.py, 20 steps, 3 alternations):
#   bash tools/gpu_r5_env_ab.sh <tag> VAR=a VAR=b ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${1:-envab}; shift; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2 3; do
  for kv in "$@"; do
    env $kv timeout -k 10 200 python -u tools/step_trace.py --mode ${MODE:-eval} --steps 20 > $OUT/${MODE:-eval}_${kv}_$rep.log 2>&1 || exit 1
    echo "== $kv: $(grep step $OUT/${MODE:-eval}_${kv}_$rep.log | tail -1)"
  done
done
