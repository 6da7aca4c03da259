# Build experimental variants of the library ON THE GPU BOX and time configs with each.
# VARIANTS="name:flags ..." (default below), CFGS="2 3 4".
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/exp
SRC=deep-multiview-depth-estimation_amd/csrc/mvs_cost_volume.hip
for v in ${VARIANTS:-base:}; do
  name=${v%%:*}; flags=$(echo ${v#*:} | tr ',' ' ')
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared $flags -o gpurun_out/exp/lib_$name.so $SRC || exit 1
  MVS_LIB_PATH=$PWD/gpurun_out/exp/lib_$name.so timeout -k 10 120 python tools/kernel_bench.py ${CFGS:-2 3 4} > gpurun_out/exp/$name.log 2>&1; rc=$?
  echo "== $name ($flags) rc=$rc"; grep cfg gpurun_out/exp/$name.log | cut -c1-150
  case $rc in 0) ;; *) exit $rc;; esac
done
rm -f gpurun_out/exp/*.so
