# LDS-staged fp32 S2 (conv_1_0): parity, layer timing, eval step A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/r6z2; mkdir -p $OUT
step() {
  local name=$1 sec=$2; shift 2
  timeout -k 10 $sec "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -20 $OUT/$name.log; exit $rc; fi
}
step parity 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "s2_lds or region_conv or channel_quad or mvsnet_end_to_end or live_regulariser or fp32_head"
tail -3 $OUT/parity.log; grep -E "^E " $OUT/parity.log | head
step lay 300 python -u tools/fp32_layers.py --only conv_1_0,conv_1_0,step,step --reps 30
grep -E " ms" $OUT/lay.log
MVS_S2_LDS=1 step lay1 300 python -u tools/fp32_layers.py --only conv_1_0,conv_1_0,step,step --reps 30
grep -E " ms" $OUT/lay1.log
exit 0
