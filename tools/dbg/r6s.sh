# prologue ref-matrix fix + chunk split for small shards: parity (split forced on), cfg timings
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/r6s; mkdir -p $OUT
step() {
  local name=$1 sec=$2; shift 2
  timeout -k 10 $sec "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -20 $OUT/$name.log; exit $rc; fi
}
MVS_CV_CSPLIT=4 step parity 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "cost_volume or golden or shard or oracle or full_size or single_view or channel_quad"
tail -3 $OUT/parity.log
for cs in 1 2 4 8; do MVS_CV_CSPLIT=$cs step k4_$cs 120 python -u tools/kernel_bench.py 4; grep '^{' $OUT/k4_$cs.log; done
MVS_BENCH_C4=1 step k235 200 python -u tools/kernel_bench.py 2 3 5
grep '^{' $OUT/k235.log
exit 0
