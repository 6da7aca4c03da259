cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/r6v5; mkdir -p $OUT
for k in s2 s1 t2; do
  MVS_TRAIN_REGION_FWD=$k timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -m gpu -q --timeout 300 --timeout-method thread -k smooth > $OUT/$k.log 2>&1; rc=$?
  echo "$k rc=$rc"; grep -E "^E .*GPU grad|passed|failed" $OUT/$k.log | head -3
  if [ $rc -gt 1 ]; then exit $rc; fi
done
exit 0
