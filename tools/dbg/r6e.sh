cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/r6e; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 -k "region or mvsnet_end_to_end or narrow" > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/fp32_layers.py > $OUT/layers_rb2.log 2>&1; rc=$?; echo "layers rb2 rc=$rc"; cat $OUT/layers_rb2.log; [ $rc -ne 0 ] && exit $rc
MVS_T2_RB=4 timeout -k 10 300 python -u tools/fp32_layers.py --only deconv_3_0,deconv_2_0,step > $OUT/layers_rb4.log 2>&1; rc=$?; echo "layers rb4 rc=$rc"; cat $OUT/layers_rb4.log; [ $rc -ne 0 ] && exit $rc
MVS_FP32_S1_LDS=0 timeout -k 10 300 python -u tools/fp32_layers.py --only step > $OUT/layers_nolds.log 2>&1; rc=$?; echo "no-lds rc=$rc"; cat $OUT/layers_nolds.log
exit $rc
