# PMC: cfg-3 warp kernel (channel-quad store) and the fp32 eval step's conv_0_0; eval-step kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; OUT=gpurun_out/r6t; mkdir -p $OUT
MVS_BENCH_C4=1 bash tools/pmc.sh r6t/pmc_cfg3 3 > $OUT/pmc_cfg3.log 2>&1; rc=$?; echo "pmc cfg3 rc=$rc"; cat $OUT/pmc_cfg3.log
[ $rc -ne 0 ] && exit $rc
python3 tools/summarize_pmc.py $OUT/pmc_cfg3 "cost_volume_staged_kernel<5" > $OUT/cfg3_pmc.json; head -c 1500 $OUT/cfg3_pmc.json
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE" bash tools/pmc_prog.sh r6t/pmc_conv0 tools/eval_steps.py --steps 3 > $OUT/pmc_conv0.log 2>&1; rc=$?; echo "pmc conv0 rc=$rc"; cat $OUT/pmc_conv0.log
[ $rc -ne 0 ] && exit $rc
python3 tools/summarize_pmc.py $OUT/pmc_conv0 "conv3d_k3_narrow_kernel<8, 1, true" > $OUT/conv0_pmc.json; cat $OUT/conv0_pmc.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/eval -o eval -- python3 tools/eval_steps.py --steps 10 > $OUT/eval.log 2>&1; echo "eval stats rc=$?"
exit 0
