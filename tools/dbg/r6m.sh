# narrow conv training kernels: parity tests, GPU train tests, cfg-2 train step
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/r6m; mkdir -p $OUT
step() {
  local name=$1 sec=$2; shift 2
  timeout -k 10 $sec "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -20 $OUT/$name.log; exit $rc; fi
}
step narrow 300 python -u -m pytest tests/test_narrow_train.py -m gpu -x -v --timeout 120 --timeout-method thread
grep -E "PASS|FAIL|Error|assert" $OUT/narrow.log | head -20
step train_tests 400 python -u -m pytest tests/test_gpu_train.py -m gpu -x -v --timeout 300 --timeout-method thread
grep -E "PASS|FAIL|Error|assert" $OUT/train_tests.log | head -20
step live 400 python -u tools/train_step_ab.py --steps 5 --prof
head -c 1200 $OUT/live.log; grep -A30 "Self CUDA" $OUT/live.log | cut -c1-72,150-215 | head -34
exit 0
