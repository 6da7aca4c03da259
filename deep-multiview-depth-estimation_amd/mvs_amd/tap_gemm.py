"""Conv3d / ConvTranspose3d with autograd as one rocBLAS GEMM per kernel tap -- the regulariser's
convolutions on the TRAINING path (train.py:97-104: MVSNet.forward under autograd, loss.backward()).

Why: MIOpen has only slow (naive) solvers for the backward passes of the regulariser's 3-D shapes --
the stride-2 convolutions with padding n//2 + 1 (config.py:20) and the full-volume transposed
convolutions -- so one cfg-2 training step took minutes.  Per tap, every convolution pass is a plain
GEMM over channels on channels-last views of the volume (hipBLASLt / rocBLAS through torch.matmul):

  conv3d forward        y[o] += x[o*s - p + t] @ W_t^T          (o, t per dim; inputs outside = 0)
         d/dx           gx[o*s - p + t] += gy[o] @ W_t
         d/dW           gW_t = sum_o gy[o]^T x[o*s - p + t]
  conv_transpose3d      y[i*s - p + t] += x[i] @ W_t            (outputs outside [0, O) dropped)
         d/dx           gx[i] += gy[i*s - p + t] @ W_t^T
         d/dW           gW_t = sum_i x[i]^T gy[i*s - p + t]

fp32 throughout (gfx950 has no reduced-precision fp32 GEMM mode to fall into); each tap's GEMM sums
over channels, taps are added in a fixed order.  Groups 1, dilation 1, no bias (the reference's
regulariser layers, model.py:76-95).
"""
import torch

_F32 = torch.float32


def _t3(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v, v)


def _conv_taps(n, out_n, k, s, p):
    """Per tap (tz, ty, tx): (output slices, input slices) of the voxels it connects in a conv3d;
    taps that connect nothing are skipped."""
    taps = []
    for tz in range(k[0]):
        for ty in range(k[1]):
            for tx in range(k[2]):
                osl, isl = [], []
                for t, d, o, pp, ss in zip((tz, ty, tx), n, out_n, p, s):
                    o0 = max(-((t - pp) // ss), 0)             # ceil((p - t) / s)
                    o1 = min((d - 1 + pp - t) // ss, o - 1)
                    if o1 < o0:
                        break
                    osl.append(slice(o0, o1 + 1))
                    isl.append(slice(o0 * ss - pp + t, o1 * ss - pp + t + 1, ss))
                if len(osl) == 3:
                    taps.append(((tz, ty, tx), tuple(osl), tuple(isl)))
    return taps


def _tconv_taps(n, out_n, k, s, p):
    """Per tap: (input slices, output slices) of a conv_transpose3d."""
    taps = []
    for tz in range(k[0]):
        for ty in range(k[1]):
            for tx in range(k[2]):
                isl, osl = [], []
                for t, d, o, pp, ss in zip((tz, ty, tx), n, out_n, p, s):
                    i0 = max(-((t - pp) // ss), 0)
                    i1 = min((o - 1 + pp - t) // ss, d - 1)
                    if i1 < i0:
                        break
                    isl.append(slice(i0, i1 + 1))
                    osl.append(slice(i0 * ss - pp + t, i1 * ss - pp + t + 1, ss))
                if len(isl) == 3:
                    taps.append(((tz, ty, tx), tuple(isl), tuple(osl)))
    return taps


def _cl(x):   # [N, C, D, H, W] -> channels-last contiguous [N, D, H, W, C]
    return x.permute(0, 2, 3, 4, 1).contiguous()


def _cf(x):   # channels-last -> [N, C, D, H, W] contiguous
    return x.permute(0, 4, 1, 2, 3).contiguous()


def _acc(dst, sl, v):
    dst[(slice(None),) + sl].add_(v)   # in place on the strided view


class _Conv3dTaps(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, padding):
        s, p, k = _t3(stride), _t3(padding), tuple(w.shape[2:])
        n = tuple(x.shape[2:])
        out_n = tuple((d + 2 * pp - kk) // ss + 1 for d, pp, kk, ss in zip(n, p, k, s))
        taps = _conv_taps(n, out_n, k, s, p)
        xc = _cl(x)
        y = torch.zeros((x.shape[0],) + out_n + (w.shape[0],), dtype=x.dtype, device=x.device)
        for (tz, ty, tx), osl, isl in taps:
            _acc(y, osl, torch.matmul(xc[(slice(None),) + isl], w[:, :, tz, ty, tx].t()))
        ctx.save_for_backward(x, w)
        ctx.geo = (n, out_n, k, s, p)
        return _cf(y)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        n, out_n, k, s, p = ctx.geo
        taps = _conv_taps(n, out_n, k, s, p)
        gyc = _cl(gy)
        gx = gw = None
        if ctx.needs_input_grad[0]:
            gxc = torch.zeros((x.shape[0],) + n + (x.shape[1],), dtype=gy.dtype, device=gy.device)
            for (tz, ty, tx), osl, isl in taps:
                _acc(gxc, isl, torch.matmul(gyc[(slice(None),) + osl], w[:, :, tz, ty, tx]))
            gx = _cf(gxc)
        if ctx.needs_input_grad[1]:
            xc = _cl(x)
            gw = torch.zeros_like(w)
            co, ci = w.shape[0], w.shape[1]
            for (tz, ty, tx), osl, isl in taps:
                g = gyc[(slice(None),) + osl].reshape(-1, co)
                gw[:, :, tz, ty, tx] = torch.matmul(g.t(), xc[(slice(None),) + isl].reshape(-1, ci))
        return gx, gw, None, None


class _ConvTranspose3dTaps(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, padding, output_padding):
        s, p, op, k = _t3(stride), _t3(padding), _t3(output_padding), tuple(w.shape[2:])
        n = tuple(x.shape[2:])
        out_n = tuple((d - 1) * ss - 2 * pp + kk + oo for d, ss, pp, kk, oo in zip(n, s, p, k, op))
        taps = _tconv_taps(n, out_n, k, s, p)
        xc = _cl(x)
        y = torch.zeros((x.shape[0],) + out_n + (w.shape[1],), dtype=x.dtype, device=x.device)
        for (tz, ty, tx), isl, osl in taps:
            _acc(y, osl, torch.matmul(xc[(slice(None),) + isl], w[:, :, tz, ty, tx]))
        ctx.save_for_backward(x, w)
        ctx.geo = (n, out_n, k, s, p)
        return _cf(y)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        n, out_n, k, s, p = ctx.geo
        taps = _tconv_taps(n, out_n, k, s, p)
        gyc = _cl(gy)
        gx = gw = None
        if ctx.needs_input_grad[0]:
            gxc = torch.zeros((x.shape[0],) + n + (x.shape[1],), dtype=gy.dtype, device=gy.device)
            for (tz, ty, tx), isl, osl in taps:
                _acc(gxc, isl, torch.matmul(gyc[(slice(None),) + osl], w[:, :, tz, ty, tx].t()))
            gx = _cf(gxc)
        if ctx.needs_input_grad[1]:
            xc = _cl(x)
            gw = torch.zeros_like(w)
            ci, co = w.shape[0], w.shape[1]
            for (tz, ty, tx), isl, osl in taps:
                gw[:, :, tz, ty, tx] = torch.matmul(xc[(slice(None),) + isl].reshape(-1, ci).t(),
                                                    gyc[(slice(None),) + osl].reshape(-1, co))
        return gx, gw, None, None, None


def conv3d(x, weight, stride=1, padding=0):
    """F.conv3d (groups 1, dilation 1, no bias) through per-tap GEMMs, differentiable."""
    return _Conv3dTaps.apply(x, weight, stride, padding)


def conv_transpose3d(x, weight, stride=1, padding=0, output_padding=0):
    """F.conv_transpose3d (groups 1, dilation 1, no bias) through per-tap GEMMs, differentiable."""
    return _ConvTranspose3dTaps.apply(x, weight, stride, padding, output_padding)


def conv_module(m, x):
    """nn.Conv3d / nn.ConvTranspose3d module ``m`` applied through the tap GEMMs."""
    if m.bias is not None or m.groups != 1 or _t3(m.dilation) != (1, 1, 1):
        return m(x)
    if isinstance(m, torch.nn.ConvTranspose3d):
        return conv_transpose3d(x, m.weight, m.stride, m.padding, m.output_padding)
    return conv3d(x, m.weight, m.stride, m.padding)
