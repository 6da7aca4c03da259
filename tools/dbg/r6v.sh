cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/r6v2; mkdir -p $OUT
step() {
  local name=$1 sec=$2; shift 2
  timeout -k 10 $sec "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -20 $OUT/$name.log; exit $rc; fi
}
step train_tests 400 python -u -m pytest tests/test_gpu_train.py -m gpu -x -v --timeout 300 --timeout-method thread
grep -E "PASS|FAIL|Error|assert" $OUT/train_tests.log | head
step taps 300 python -u tools/train_step_ab.py --steps 3
grep '^{' $OUT/taps.log | cut -c1-260
exit 0
