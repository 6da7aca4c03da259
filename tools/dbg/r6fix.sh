# fused head built without packed fp32: stress at the bench geometry, then the head tests and smoke
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/r6fix; mkdir -p $OUT
HEAD_STRESS_CFGS="4,3,192,128,160;4,2,192,128,160;1,3,100,36,44" STRESS_N=300 bash tools/dbg/stress_r6.sh r6fix deep-multiview-depth-estimation_amd/mvs_amd/libmvs_cost_volume.so || exit $?
timeout -k 10 300 python -u -m pytest tests/test_cv_head.py -m gpu -v --timeout 120 --timeout-method thread -rxX > $OUT/pytest_cv_head.log 2>&1; rc=$?; tail -4 $OUT/pytest_cv_head.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1; rc=$?; tail -1 $OUT/smoke.log; exit $rc
