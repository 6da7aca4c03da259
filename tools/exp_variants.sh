# Build experimental variants of the library ON THE GPU BOX and time configs with each.
# VARIANTS="name:flag1,flag2 ..." (default: base), CFGS="2 3 4".
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/exp
for v in ${VARIANTS:-base:}; do
  name=${v%%:*}; flags=${v#*:}
  python -c "import sys; sys.path.insert(0, 'deep-multiview-depth-estimation_amd'); from mvs_amd import _build; _build.build_library(force=True, extra_flags=[f for f in '$flags'.split(',') if f], output='/tmp/lib_$name.so')" || exit 1
  MVS_LIB_PATH=/tmp/lib_$name.so timeout -k 10 120 python tools/kernel_bench.py ${CFGS:-2 3 4} > gpurun_out/exp/$name.log 2>&1; rc=$?
  echo "== $name ($flags) rc=$rc"; grep cfg gpurun_out/exp/$name.log | cut -c1-150
  case $rc in 0) ;; *) exit $rc;; esac
done
