# Round-2 first look: live-step kernel breakdown (eval), train-mode and grad step times, channels-last probe.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r2a_eval" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/step_trace.py" --mode eval > gpurun_out/r2a_eval.log 2>&1
rc=$?; echo "eval prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/step_trace.py --mode train --steps 3 > gpurun_out/r2a_train.log 2>&1; rc=$?; echo "train rc=$rc"; cat gpurun_out/r2a_train.log | tail -2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/step_trace.py --mode grad --steps 3 --batch 2 > gpurun_out/r2a_grad.log 2>&1; rc=$?; echo "grad rc=$rc"; tail -2 gpurun_out/r2a_grad.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/e2e_breakdown.py > gpurun_out/r2a_e2e.log 2>&1; rc=$?; echo "e2e rc=$rc"; grep "step ms" gpurun_out/r2a_e2e.log
exit $rc
