# Channel sweep of the fused kernel (set-up vs per-chunk cost) for library variants.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/exp
for v in ${VARIANTS:-base:}; do
  name=${v%%:*}; flags=${v#*:}
  python -c "import sys; sys.path.insert(0, 'deep-multiview-depth-estimation_amd'); from mvs_amd import _build; _build.build_library(force=True, extra_flags=[f for f in '$flags'.split(',') if f], output='/tmp/lib_$name.so')" || exit 1
  for c in 4 8 16 32; do
    MVS_BENCH_C=$c MVS_LIB_PATH=/tmp/lib_$name.so timeout -k 10 120 python tools/kernel_bench.py 2 > gpurun_out/exp/${name}_c$c.log 2>&1; rc=$?
    echo "== $name C=$c rc=$rc $(grep cfg gpurun_out/exp/${name}_c$c.log | cut -c1-110)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
