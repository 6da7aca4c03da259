cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/r6v7; mkdir -p $OUT
step() {
  local name=$1 sec=$2; shift 2
  timeout -k 10 $sec "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -20 $OUT/$name.log; exit $rc; fi
}
step tests 500 python -u -m pytest tests/test_narrow_train.py tests/test_gpu_train.py -m gpu -x -v --timeout 300 --timeout-method thread
grep -E "PASS|FAIL|Error|^E " $OUT/tests.log | head -20
step hip 300 python -u tools/train_step_ab.py --steps 3
grep '^{' $OUT/hip.log | cut -c1-230
MVS_TRAIN_REGION_FWD=hip step allhip 300 python -u tools/train_step_ab.py --steps 3
grep '^{' $OUT/allhip.log | cut -c1-230
exit 0
