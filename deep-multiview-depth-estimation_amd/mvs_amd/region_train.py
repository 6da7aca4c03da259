"""The live-region regulariser's region convolutions under autograd (train.py:97-104 through
CostVolumeReg.forward_live_train's torch layers) with their FORWARD on the HIP region kernels
(csrc/conv3d_region.hip: fp32 MFMA, the eval path's kernels without the BN epilogue) and the per-tap-GEMM
backward (tap_gemm.conv3d_backward / conv_transpose3d_backward: the same box geometry as tap_gemm's
conv3d_box / conv_transpose3d_box).  The tap GEMMs accumulate every tap's product into the output in HBM
(27 read-modify-write passes over it); the region kernels keep the accumulators in registers.

  stride-2 conv_k_0 (model.py:101-107, stacked 32 -> 16 + 32 + 64 over R2)  mode S2, one launch per layer
  stride-1 conv_k_1 (model.py:108-113, on R1 from the padded R2 crop)         mode S1
  transposed deconv_3_0 / deconv_2_0 (model.py:117-120, the full box from M)  mode T2
MVS_TRAIN_REGION_FWD selects which (enabled())."""
import os

import torch

from . import tap_gemm

S2_SPLITS = (16, 32, 64)   # conv_1_0, conv_2_0, conv_3_0 output channels (the stacked S2 order)
S1_CHANNELS = (16, 32, 64)
T2_SHAPES = ((64, 32), (32, 16))   # (c_in, c_out) of deconv_3_0, deconv_2_0


def enabled(x, kind=None):
    """kind "s2" / "s1" / "t2"; MVS_TRAIN_REGION_FWD: a comma list of kinds (default "s1,t2"), "hip" (all)
    or "taps" (none).  The stride-2 forward stays on the tap GEMMs by default: with it on the HIP kernel
    test_gpu_train.py::test_train_mode_autograd_chain_smooth_loss's deconv_1_0 weight gradient lands 2.8x
    the CPU fp32 error from float64 (0.0074 against 0.0027)."""
    v = os.environ.get("MVS_TRAIN_REGION_FWD", "s1,t2")
    on = v == "hip" or (kind is not None and kind in v.split(","))
    return on and x.is_cuda and x.dtype == torch.float32 and torch.is_grad_enabled()


def _region_w(w):      # Conv3d weight [co, ci, 3, 3, 3] -> [27][co][ci]
    return w.detach().permute(2, 3, 4, 0, 1).reshape(27, w.shape[0], w.shape[1]).contiguous()


def _region_wt(w):     # ConvTranspose3d weight [ci, co, 3, 3, 3] -> [27][co][ci]
    return w.detach().permute(2, 3, 4, 1, 0).reshape(27, w.shape[1], w.shape[0]).contiguous()


def _cf(t):            # channels-last [B, d, h, w, C] -> logical NCDHW view
    return t.permute(0, 4, 1, 2, 3)


class _S2Box(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, out_reg, pad, pad_lo, splits):
        from .ops import CONV_S2, conv3d_region
        n = list(x.shape[2:])
        org, size = [lo for lo, _ in out_reg], [hi - lo + 1 for lo, hi in out_reg]
        xc = x.contiguous()
        ys, c0 = [], 0
        for co in splits:
            ys.append(conv3d_region(xc, None, _region_w(w[c0:c0 + co]), CONV_S2, n, org, size, None, None, list(pad)))
            c0 += co
        ctx.save_for_backward(x, w)
        ctx.geo = (tuple(pad_lo), tuple(size))
        return _cf(torch.cat(ys, -1) if len(ys) > 1 else ys[0])

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx, gw = tap_gemm.conv3d_backward(x, w, 2, ctx.geo[0], ctx.geo[1], gy, ctx.needs_input_grad[0],
                                          ctx.needs_input_grad[1])
        return gx, gw, None, None, None, None


class _S1Valid(torch.autograd.Function):
    """conv3d(xin, w) with padding 0 (xin: the zero-padded crop of _conv_s1_region)."""

    @staticmethod
    def forward(ctx, xin, w):
        from .ops import CONV_S1, conv3d_region
        L = list(xin.shape[2:])
        out = [d - 2 for d in L]
        y = conv3d_region(xin.permute(0, 2, 3, 4, 1).contiguous(), None, _region_w(w), CONV_S1, L, [1, 1, 1], out,
                          [0, 0, 0], L, None)
        ctx.save_for_backward(xin, w)
        ctx.out = tuple(out)
        return _cf(y)

    @staticmethod
    def backward(ctx, gy):
        xin, w = ctx.saved_tensors
        gx, gw = tap_gemm.conv3d_backward(xin, w, 1, 0, ctx.out, gy, ctx.needs_input_grad[0], ctx.needs_input_grad[1])
        return gx, gw


class _T2Box(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, x_reg, out_reg, pad, dims, crop):
        from .ops import CONV_T2, conv3d_region
        org, size = [lo for lo, _ in out_reg], [hi - lo + 1 for lo, hi in out_reg]
        xorg, xsize = [lo for lo, _ in x_reg], [hi - lo + 1 for lo, hi in x_reg]
        y = conv3d_region(x.permute(0, 2, 3, 4, 1).contiguous(), None, _region_wt(w), CONV_T2, list(dims), org, size,
                          xorg, xsize, list(pad))
        ctx.save_for_backward(x, w)
        ctx.geo = (tuple(crop), tuple(size))
        return _cf(y)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx, gw = tap_gemm.conv_transpose3d_backward(x, w, 2, ctx.geo[0], ctx.geo[1], gy, ctx.needs_input_grad[0],
                                                    ctx.needs_input_grad[1])
        return gx, gw, None, None, None, None, None


def s2_box(x, w, out_reg, pad, pad_lo, splits):
    return _S2Box.apply(x, w, out_reg, pad, pad_lo, splits)


def s1_valid(xin, w):
    return _S1Valid.apply(xin, w)


def t2_box(x, w, x_reg, out_reg, pad, dims, crop):
    return _T2Box.apply(x, w, x_reg, out_reg, pad, dims, crop)
