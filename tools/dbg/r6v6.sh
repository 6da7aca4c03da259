cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/r6v6; mkdir -p $OUT
timeout -k 10 300 python -u tools/dbg/s2_acc.py > $OUT/acc.log 2>&1; rc=$?; echo "rc=$rc"; cat $OUT/acc.log | grep -v amdgpu; exit $rc
