cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/r6g; mkdir -p $OUT
for v in "0 0" "1 0" "0 1" "1 1" "0 0"; do set -- $v
MVS_CHAIN_PRIO=$1 MVS_FP32_LEVELS=$2 timeout -k 10 300 python -u tools/fp32_layers.py --only step,step --reps 30 > $OUT/step_p$1_l$2.log 2>&1; rc=$?; echo "prio $1 levels $2 rc=$rc"; grep step $OUT/step_p$1_l$2.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
