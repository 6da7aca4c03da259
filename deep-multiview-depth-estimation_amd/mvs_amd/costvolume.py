"""Drop-in for ``scripts/costvolume.py`` plus the fused warp + variance entry point.

``assemble_cost_volume(warped, n_views)`` keeps the reference signature (:3-16) and runs the
variance in ``mvs::assemble_cost_volume`` (HIP).

``warp_and_assemble_cost_volume(...)`` replaces ``model.py:177-181`` (homography_warping followed by
assemble_cost_volume) with ONE fused HIP kernel (``mvs::cost_volume``): every view is gathered and
the two-pass variance is accumulated in registers, so the B*V x C x D x h x w warped volume is never
written; ``d_begin``/``d_count`` select a depth shard for the multi-GPU path.

``DeferredCostVolume`` (``warp_and_assemble_cost_volume(..., deferred=True)``) goes one step further
(SURVEY.md §8 f3): it carries the INPUTS of the cost volume to ``CostVolumeReg``, whose eval path forms
the variance on chip inside its first two convolutions (``mvs::cost_volume_head``) -- the volume is
never written; any other consumer calls ``.materialize()``.
"""
import torch

from . import ops
from .config import D_NUM, D_SCALE
from .homography import depth_hypotheses, reference_indices


def assemble_cost_volume(warped_feature_maps, n_views: int):
    return ops.assemble_cost_volume_op(warped_feature_maps, int(n_views))


class DeferredCostVolume:
    """The cost volume of ``model.py:177-181`` (homography_warping + assemble_cost_volume), NOT formed:
    the features, cameras and depth planes it is a function of.  ``CostVolumeReg.forward`` consumes it
    where it is formed (the fused head kernel, csrc/cv_head.hip: variance + conv_0_0 + conv_1_0 on chip);
    ``materialize()`` forms the reference tensor [B, C, D, h, w] fp32 (mvs::cost_volume) for any other
    consumer.  ``shape`` / ``dtype`` / ``device`` describe that tensor."""

    def __init__(self, K_batch, R_batch, T_batch, d_min, d_int, feature_maps, batch_size, n_views,
                 d_num, d_scale):
        self.K, self.R, self.T, self.d_min, self.d_int = K_batch, R_batch, T_batch, d_min, d_int
        self.feature_maps = feature_maps
        self.batch_size, self.n_views = int(batch_size), int(n_views)
        self.d_num, self.d_scale = int(d_num), float(d_scale)
        _, c, h, w = feature_maps.shape
        self.shape = torch.Size((self.batch_size, c, self.d_num, h, w))
        self.dtype = torch.float32
        self.device = feature_maps.device
        self.is_cuda = feature_maps.is_cuda

    def dim(self):
        return 5

    def head(self, w0, bn0, w1, bn1, pad, y1_origin, y1_size, scv_lo, scv_hi):
        """ops.cost_volume_head on these inputs: (y0, y1, BoundCostVolume of the scv box)."""
        y0, y1, scv, absmax = ops.cost_volume_head(
            self.feature_maps, self.K, self.R, self.T, self.d_min, self.d_int, self.batch_size, self.n_views,
            0, self.d_num, self.d_scale, w0, *bn0, w1, *bn1, list(pad), list(y1_origin), list(y1_size),
            list(scv_lo), list(scv_hi))
        return y0, y1, ops.BoundCostVolume(scv, absmax, scv_lo, self.shape[2:]) if scv.dim() == 6 else None

    def materialize(self):
        cv, _ = ops.cost_volume(self.feature_maps, self.K, self.R, self.T, self.d_min, self.d_int,
                                self.batch_size, self.n_views, 0, self.d_num, self.d_scale)
        return cv


def warp_and_assemble_cost_volume(K_batch, R_batch, T_batch, d_min, d_int, feature_maps,
                                  batch_size, n_views, d_num=D_NUM, d_scale=D_SCALE,
                                  d_begin=0, d_count=None, cv_dtype=torch.float32, channel_quads=False,
                                  split=False, deferred=False):
    """-> (cv [B, C, d_count, h, w], d_batch_0 [B, d_num, 1, 1], ref_idx_0 [B] CPU int64).

    ``cv_dtype=torch.bfloat16`` (opt-in) returns the fp32 variance rounded to
    bf16 in the kernel's store (half the write); the default fp32 is the reference's.
    ``channel_quads=True`` (inference) returns the same values in the channel-quad layout
    [B, C/4, d_count, h, w, 4] that CostVolumeReg's HIP path reads 16 (fp32) or 8 (bf16) bytes at a
    time; fp32 comes as ops.BoundCostVolume (the volume with its bound words).  ``split=True`` (with
    channel_quads, fp32): the SPLIT cost volume (int32 elements holding the fp16 hi / lo parts the
    split-fp16 regulariser kernels read, csrc/split.h).  ``deferred=True`` (fp32, whole depth range):
    a DeferredCostVolume -- nothing is computed until CostVolumeReg consumes it."""
    if d_count is None:
        d_count = d_num - d_begin
    if d_begin < 0 or d_count <= 0 or d_begin + d_count > d_num:
        raise ValueError("depth shard [%d, %d) outside [0, %d)" % (d_begin, d_begin + d_count, d_num))
    device = feature_maps.device
    d_batch_0 = depth_hypotheses(d_min, d_int, d_num, d_scale).to(device)
    if deferred:
        if cv_dtype != torch.float32 or d_begin != 0 or d_count != d_num:
            raise ValueError("a deferred cost volume is fp32 over the whole depth range")
        return (DeferredCostVolume(K_batch, R_batch, T_batch, d_min, d_int, feature_maps, batch_size, n_views,
                                   d_num, d_scale), d_batch_0, reference_indices(batch_size, n_views))
    if channel_quads:
        if cv_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("the channel-quad cost volume is fp32 or bf16, got %s" % (cv_dtype,))
        args = (feature_maps, K_batch, R_batch, T_batch, d_min, d_int, int(batch_size), int(n_views),
                int(d_begin), int(d_count), float(d_scale))
        if cv_dtype == torch.float32:
            # with its bound words (max |feat|), the split-fp16 regulariser kernels' scale
            # (ops.conv3d_k3_split, ops.conv_s2_split)
            cv = ops.BoundCostVolume(*(ops.cost_volume_c4_split if split else ops.cost_volume_c4_absmax)(*args))
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
