cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/exp
SRC=deep-multiview-depth-estimation_amd/csrc/mvs_cost_volume.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -DMVS_EXP_PG=4 -DMVS_EXP_NO_STORE -DMVS_EXP_NO_GATHER -DMVS_EXP_NO_STAGE -o /tmp/skel.so $SRC || exit 1
MVS_LIB_PATH=/tmp/skel.so bash tools/pmc.sh pmc_skel 2
