cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/r6t2; mkdir -p $OUT
timeout -k 10 400 python -u tools/train_step_ab.py --steps 3 --prof --ops > $OUT/ops.log 2>&1; rc=$?; echo "rc=$rc"; exit $rc
