"""The regulariser's two narrow full-volume convolutions under autograd (train.py:97-104: loss.backward
through model.py:101 conv_0_0, Conv3d(32, 8, 3, padding 1), and model.py:124 conv_out, Conv3d(8, 1, 3,
padding 1)) on the HIP kernels, fp32:

  forward        y  = conv3d(x, w)              mvs_conv3d_k3_fwd (csrc/conv3d_narrow.hip)
  d/dx           gx = conv3d(gy, w~)            the same kernel, w~[ci][co] = w[co][ci] flipped in every
                                                tap dim, 8 input-gradient channels per launch
  d/dw           gw[co][ci][t] = sum gy x(t)    mvs_conv3d_k3_wgrad (csrc/conv3d_wgrad.hip, f32 MFMA)

They replace the per-tap rocBLAS GEMMs (tap_gemm.py), which stream the full volume once per tap in each
pass (cfg 2: 112 ms for conv_0_0's forward + backward, 106 ms for conv_out's; tools/train_layers.py)."""
import os

import torch

from . import ops


def applies(conv, x):
    """conv (an nn.Conv3d of the regulariser) on x runs here: a HIP fp32 NCDHW input under autograd,
    kernel 3, stride 1, padding 1, no bias, (c_in, c_out) with a weight-gradient kernel
    (ops.WGRAD_SHAPES), MVS_TRAIN_NARROW not 0."""
    w = conv.weight
    return (os.environ.get("MVS_TRAIN_NARROW", "1") != "0" and x.is_cuda and x.dtype == torch.float32
            and x.dim() == 5 and not torch.is_autocast_enabled() and conv.bias is None and conv.groups == 1
            and tuple(w.shape[2:]) == (3, 3, 3) and tuple(conv.stride) == (1, 1, 1)
            and tuple(conv.padding) == (1, 1, 1) and tuple(conv.dilation) == (1, 1, 1)
            and (w.shape[1], w.shape[0]) in ops.WGRAD_SHAPES and w.shape[1] % 8 == 0)


def _data_weight(w):
    """The input gradient's weight: w~[ci][co][t] = w[co][ci][26 - t]."""
    return w.flip(2, 3, 4).transpose(0, 1).contiguous()


class _NarrowConv3d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return ops.conv3d_k3(x.contiguous(), w)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy = gy.contiguous()
        gx = gw = None
        if ctx.needs_input_grad[0]:
            wt = _data_weight(w.detach())
            parts = [ops.conv3d_k3(gy, wt[g:g + 8]) for g in range(0, wt.shape[0], 8)]
            gx = parts[0] if len(parts) == 1 else torch.cat(parts, 1)
        if ctx.needs_input_grad[1]:
            gw = ops.conv3d_k3_wgrad(x, gy)
        return gx, gw


def conv3d(conv, x):
    """conv(x) for an nn.Conv3d that applies(), differentiable in x and conv.weight."""
    return _NarrowConv3d.apply(x, conv.weight)
