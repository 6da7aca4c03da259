# fused fp32 head: parity tests, the round-6 pending checks, layer timings, a short bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/r6i; mkdir -p $OUT
step() {   # step NAME SECONDS CMD...: stop the call on a fault / abort / time limit (test failures go on)
  local name=$1 sec=$2; shift 2
  timeout -k 10 $sec "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -20 $OUT/$name.log; exit $rc; fi
}
step head 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "fp32_head or mvsnet_end_to_end or rccl or pipelined or sharded"
grep -E "PASS|FAIL|Error|assert" $OUT/head.log | head -30
step layers 300 python -u tools/fp32_layers.py --only conv_0_0,conv_1_0,conv_head,step,step --reps 30
grep -E "ms|equal" $OUT/layers.log
MVS_FP32_HEAD=0 step layers_nohead 300 python -u tools/fp32_layers.py --only step,step --reps 30
grep ms $OUT/layers_nohead.log
step bench 400 python -u bench.py --steps 20 --warmup 5
tail -c 3000 $OUT/bench.log
exit 0
