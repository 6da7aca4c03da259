# A/B of the narrow-conv kernel variants (-D flags) on the regulariser layer timings.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "narrow or live or end_to_end or region_deconv" -q --timeout 200 --timeout-method thread > gpurun_out/pt_conv2.log 2>&1; rc=$?; tail -3 gpurun_out/pt_conv2.log; [ $rc -ne 0 ] && exit $rc
for v in ${VARIANTS:-nr1:-DMVS_EXP_CONV_NR=1 nr2:-DMVS_EXP_CONV_NR=2}; do
  name=${v%%:*}; flags=${v#*:}
  python -c "import sys; sys.path.insert(0, 'deep-multiview-depth-estimation_amd'); from mvs_amd import _build; _build.build_library(force=True, extra_flags=[f for f in '$flags'.split(',') if f], output='/tmp/lib_$name.so')" > /dev/null 2>&1 || exit 1
  echo "== $name"; MVS_LIB_PATH=/tmp/lib_$name.so timeout -k 10 200 python tools/reg_layers.py 2>&1 | grep -E "HIP|whole"
done
timeout -k 10 200 python tools/e2e_breakdown.py 2>&1 | grep "live step ms" | head -1
