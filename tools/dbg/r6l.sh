cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/r6l; mkdir -p $OUT
timeout -k 10 900 python -u tools/train_layers.py --reps 2 > $OUT/layers.log 2>&1; rc=$?; echo "rc=$rc"; cat $OUT/layers.log | grep -v amdgpu.ids; exit $rc
