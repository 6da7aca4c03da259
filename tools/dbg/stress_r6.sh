# fused-head repeatability under library variants: bash tools/dbg/stress_r6.sh <tag> <lib>...
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/$1; shift; mkdir -p $OUT
export HEAD_STRESS_CFGS="${HEAD_STRESS_CFGS:-1,3,48,28,64;4,3,192,128,160;4,2,192,128,160}" HEAD_STRESS_SHOW=2
for lib in "$@"; do n=$(basename $lib .so)
  MVS_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u tools/dbg/head_stress.py ${STRESS_N:-20} bn > $OUT/$n.log 2>&1; rc=$?
  echo "$n rc=$rc"; grep -E "^cfg" $OUT/$n.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
