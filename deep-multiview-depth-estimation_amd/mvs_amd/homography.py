"""Drop-in for ``scripts/homography.py`` (reference ``homography_warping``, :6-92).

Same name, arguments, defaults, return tuple and devices as the reference:

    homography_warping(K_batch, R_batch, T_batch, d_min, d_int, feature_maps,
                       batch_size, n_views, d_num=D_NUM)
        -> (warped [B*V, C, D, h, w] on the feature device,
            d_batch_0 [B, D, 1, 1] on the feature device,
            ref_idx_0 [B] int64 on the CPU)

The warp runs in ``mvs::homography_warp`` (HIP, gfx950): per-(image, plane) sampling matrices in
fp64, then one bilinear-gather kernel writing every plane directly -- no per-plane Python loop,
no O(D^2) ``torch.cat`` growth (homography.py:83-90).  Models should prefer the fused
``costvolume.warp_and_assemble_cost_volume``, which never materialises this warped volume.
"""
import torch

from . import ops
from .config import D_NUM, D_SCALE


def depth_hypotheses(d_min, d_int, d_num, d_scale=D_SCALE):
    """homography.py:24-26: d_batch_0 = d_min + D_SCALE * d_int * k, shape [B, D, 1, 1].  fp32
    inference on the GPU with the data loader's [B, 1, 1, 1] shapes: one HIP launch (ops.depth_hypotheses,
    bit-equal to the expression below)."""
    if (d_min.is_cuda and d_int.is_cuda and d_min.dtype == torch.float32 and d_int.dtype == torch.float32
            and not torch.is_grad_enabled() and d_min.dim() == 4 and tuple(d_min.shape[1:]) == (1, 1, 1)
            and tuple(d_int.shape) == tuple(d_min.shape)):
        return ops.depth_hypotheses(d_min, d_int, d_num, d_scale)
    d_num_tensor = torch.arange(d_num, device=d_min.device).reshape(1, d_num, 1, 1)
    return d_min + d_scale * d_int * d_num_tensor


def reference_indices(batch_size, n_views):
    """homography.py:29: one reference view per sample, index b * n_views (CPU int64)."""
    return torch.arange(0, batch_size * n_views, n_views)


def homography_warping(K_batch, R_batch, T_batch, d_min, d_int, feature_maps, batch_size,
                       n_views, d_num=D_NUM, d_scale=D_SCALE):
    device = feature_maps.device
    d_batch_0 = depth_hypotheses(d_min, d_int, d_num, d_scale).to(device)
    warped = ops.homography_warp(feature_maps, K_batch, R_batch, T_batch, d_min, d_int,
                                 int(batch_size), int(n_views), 0, int(d_num), float(d_scale))
    return warped, d_batch_0, reference_indices(batch_size, n_views)
