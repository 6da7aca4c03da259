# per-config warp-kernel rocprof stats (kernel_configs legs): cfg 2/3/5 channel-quad store, cfg 4 shard NCDHW
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; OUT=gpurun_out/r6r; mkdir -p $OUT
for c in 2 3 4 5; do
  q=1; [ $c = 4 ] && q=0
  MVS_BENCH_C4=$q timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/cfg$c -o cfg$c -- python3 tools/kernel_bench.py $c > $OUT/cfg$c.log 2>&1; rc=$?
  echo "cfg$c rc=$rc"; grep '^{' $OUT/cfg$c.log
  if [ $rc -ne 0 ]; then tail -5 $OUT/cfg$c.log; exit $rc; fi
done
find $OUT -name "*kernel_stats.csv" | head
exit 0
