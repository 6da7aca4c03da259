"""Drop-in for ``scripts/costvolume.py`` plus the fused warp + variance entry point.

``assemble_cost_volume(warped, n_views)`` keeps the reference signature (:3-16) and runs the
variance in ``mvs::assemble_cost_volume`` (HIP).

``warp_and_assemble_cost_volume(...)`` replaces ``model.py:177-181`` (homography_warping followed by
assemble_cost_volume) with ONE fused HIP kernel (``mvs::cost_volume``): every view is gathered and
the two-pass variance is accumulated in registers, so the B*V x C x D x h x w warped volume is never
written; ``d_begin``/``d_count`` select a depth shard for the multi-GPU path.
"""
import torch

from . import ops
from .config import D_NUM, D_SCALE
from .homography import depth_hypotheses, reference_indices


def assemble_cost_volume(warped_feature_maps, n_views: int):
    return ops.assemble_cost_volume_op(warped_feature_maps, int(n_views))


def warp_and_assemble_cost_volume(K_batch, R_batch, T_batch, d_min, d_int, feature_maps,
                                  batch_size, n_views, d_num=D_NUM, d_scale=D_SCALE,
                                  d_begin=0, d_count=None, cv_dtype=torch.float32, channel_quads=False,
                                  split=False):
    """-> (cv [B, C, d_count, h, w], d_batch_0 [B, d_num, 1, 1], ref_idx_0 [B] CPU int64).

    ``cv_dtype=torch.bfloat16`` (opt-in) returns the fp32 variance rounded to
    bf16 in the kernel's store (half the write); the default fp32 is the reference's.
    ``channel_quads=True`` (inference) returns the same values in the channel-quad layout
    [B, C/4, d_count, h, w, 4] that CostVolumeReg's HIP path reads 16 (fp32) or 8 (bf16) bytes at a
    time.  ``split=True`` (with channel_quads, fp32): the SPLIT cost volume (int32 elements holding
    the fp16 hi / lo parts the split-fp16 regulariser kernels read, csrc/split.h), its bound words
    registered beside it (ops.cv_bound)."""
    if d_count is None:
        d_count = d_num - d_begin
    if d_begin < 0 or d_count <= 0 or d_begin + d_count > d_num:
        raise ValueError("depth shard [%d, %d) outside [0, %d)" % (d_begin, d_begin + d_count, d_num))
    device = feature_maps.device
    d_batch_0 = depth_hypotheses(d_min, d_int, d_num, d_scale).to(device)
    if channel_quads:
        if cv_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("the channel-quad cost volume is fp32 or bf16, got %s" % (cv_dtype,))
        args = (feature_maps, K_batch, R_batch, T_batch, d_min, d_int, int(batch_size), int(n_views),
                int(d_begin), int(d_count), float(d_scale))
        if cv_dtype == torch.float32:
            # with its bound words (max |feat|), registered beside the tensor for the split-fp16
            # regulariser kernels (ops.conv3d_k3_split, ops.conv_s2_split)
            cv, absmax = (ops.cost_volume_c4_split if split else ops.cost_volume_c4_absmax)(*args)
            ops.register_cv_bound(cv, absmax)
        else:
            cv = ops.cost_volume_c4_bf16(*args)
        return cv, d_batch_0, reference_indices(batch_size, n_views)
    if cv_dtype == torch.float32:
        op = ops.cost_volume
    elif cv_dtype == torch.bfloat16:
        op = ops.cost_volume_bf16
    else:
        raise ValueError("cv_dtype must be torch.float32 or torch.bfloat16, got %s" % (cv_dtype,))
    cv, _ = op(feature_maps, K_batch, R_batch, T_batch, d_min, d_int, int(batch_size), int(n_views),
               int(d_begin), int(d_count), float(d_scale))
    return cv, d_batch_0, reference_indices(batch_size, n_views)
