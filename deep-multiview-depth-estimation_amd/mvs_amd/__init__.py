"""mvs_amd -- MI355X-native MVSNet cost-volume path (drop-in for bcollico/Deep-Multiview-Depth-
Estimation's scripts/homography.py, costvolume.py, depthmap.py and model.MVSNet).

HIP kernels live in ../csrc (libmvs_cost_volume.so, C ABI in ../../include/mvs_cost_volume.h).
"""
from . import _lib, config, ops  # noqa: F401
from .costvolume import assemble_cost_volume, warp_and_assemble_cost_volume  # noqa: F401
from .depthmap import extract_depth_map  # noqa: F401
from .homography import homography_warping  # noqa: F401

__all__ = ["homography_warping", "assemble_cost_volume", "warp_and_assemble_cost_volume",
           "extract_depth_map", "config", "ops"]
