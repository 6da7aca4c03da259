#!/bin/bash
# PMC of both split kernels (pre-split input) on the cfg-2 volume.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_r3p.sh r3r_s2 conv_1_0_split conv_s2_split_kernel || exit $?
bash tools/gpu_r3p.sh r3r_c0 conv_0_0_split conv0_split_kernel
