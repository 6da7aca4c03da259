# Round 2: channels-last probe + the full bench
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 tools/cl_probe.py ncdhw > gpurun_out/r2f_cl_ncdhw.log 2>&1; rc=$?; echo "ncdhw rc=$rc"; grep "live step" gpurun_out/r2f_cl_ncdhw.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r2f_cl" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/cl_probe.py" cl > gpurun_out/r2f_cl.log 2>&1; rc=$?; echo "cl rc=$rc"; grep "live step" gpurun_out/r2f_cl.log; [ $rc -ne 0 ] && exit $rc
s=$(date +%s); timeout -k 10 900 python bench.py > gpurun_out/r2f_bench.log 2> gpurun_out/r2f_bench.err; rc=$?; echo "bench rc=$rc wall=$(( $(date +%s) - s ))s"; tail -1 gpurun_out/r2f_bench.log | cut -c1-600
exit $rc
