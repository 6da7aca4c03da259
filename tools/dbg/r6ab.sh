# A/B: deconv_2_0 with four row blocks (default now) vs two (MVS_T2_RB=2): eval step, train step, region tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/r6ab2; mkdir -p $OUT
run() { local name=$1; shift; env "$@" timeout -k 10 200 python -u tools/fp32_layers.py --only step,step,deconv_3_0,deconv_2_0 --reps 30 > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep ' ms' $OUT/$name.log | awk '{print $2}' | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc; return 0; }
run rb4 MVS_X=0
run rb2 MVS_T2_RB=2
run rb4b MVS_X=0
timeout -k 10 300 python -u tools/train_step_ab.py --steps 5 > $OUT/train_rb4.log 2>&1 || exit $?
MVS_T2_RB=2 timeout -k 10 300 python -u tools/train_step_ab.py --steps 5 > $OUT/train_rb2.log 2>&1 || exit $?
tail -3 $OUT/train_rb4.log; tail -3 $OUT/train_rb2.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "region or deconv or train or live" > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; exit $rc
