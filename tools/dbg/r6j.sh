# fused fp32 head variants (tools/exp_libs: packed / scalar FMAs, channel-plane pad): layer timings
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/r6j; mkdir -p $OUT
step() {
  local name=$1 sec=$2; shift 2
  timeout -k 10 $sec "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -20 $OUT/$name.log; exit $rc; fi
}
for v in pk sc sccp pkcp; do
  MVS_LIB_PATH=tools/exp_libs/lib_$v.so step $v 240 python -u tools/fp32_layers.py --only conv_0_0,conv_1_0,conv_head,conv_head,step --reps 30
  grep -E "ms|equal" $OUT/$v.log
done
exit 0
