"""Test-side fp32 reference of Conv3d / ConvTranspose3d as one GEMM per kernel tap (rocBLAS through
torch.matmul on a HIP device), independent of the HIP kernels under test AND of MIOpen.

Why: at cfg 5 (296x400 features, D=256) MIOpen has only slow solvers for several of the
regulariser's shapes (the stride-2 convs with padding n//2+1 ran ~7 minutes per forward); a tap
GEMM needs no solver search and runs in well under a second per layer.

conv3d:            out[o] = sum_t x[o*s - p + t] @ w[:, :, t]^T  (o, t per dim; x outside = 0)
conv_transpose3d:  out[i*s - p + t] += x[i] @ w[:, :, t]         (outputs outside [0, O) dropped)
Each tap is a [voxels, C_in] x [C_in, C_out] fp32 matmul on channels-last views; taps are summed in
a fixed order (z, y, x).  Only what the reference model uses is supported (groups 1, dilation 1).
"""
import contextlib

import torch
import torch.nn.functional as F


def _t3(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v, v)


def conv3d_taps(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1):
    assert groups == 1 and _t3(dilation) == (1, 1, 1), "tap reference: groups 1, dilation 1 only"
    s, p, k = _t3(stride), _t3(padding), tuple(weight.shape[2:])
    n = tuple(x.shape[2:])
    out_n = tuple((d + 2 * pp - kk) // ss + 1 for d, pp, kk, ss in zip(n, p, k, s))
    xc = x.permute(0, 2, 3, 4, 1)                              # [N, D, H, W, Ci] view
    out = torch.zeros((x.shape[0],) + out_n + (weight.shape[0],), dtype=x.dtype, device=x.device)
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
                if len(osl) < 3:
                    continue
                xs = xc[:, isl[0], isl[1], isl[2], :]
                out[:, osl[0], osl[1], osl[2], :] += torch.matmul(xs, weight[:, :, tz, ty, tx].t())
    if bias is not None:
        out += bias
    return out.permute(0, 4, 1, 2, 3).contiguous()


def conv_transpose3d_taps(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1,
                          dilation=1):
    assert groups == 1 and _t3(dilation) == (1, 1, 1), "tap reference: groups 1, dilation 1 only"
    s, p, op, k = _t3(stride), _t3(padding), _t3(output_padding), tuple(weight.shape[2:])
    n = tuple(x.shape[2:])
    out_n = tuple((d - 1) * ss - 2 * pp + kk + oo for d, ss, pp, kk, oo in zip(n, s, p, k, op))
    xc = x.permute(0, 2, 3, 4, 1)
    out = torch.zeros((x.shape[0],) + out_n + (weight.shape[1],), dtype=x.dtype, device=x.device)
    for tz in range(k[0]):
        for ty in range(k[1]):
            for tx in range(k[2]):
                osl, isl = [], []
                for t, d, o, pp, ss in zip((tz, ty, tx), n, out_n, p, s):
                    i0 = max(-((t - pp) // ss), 0)             # first input with i*s - p + t >= 0
                    i1 = min((o - 1 + pp - t) // ss, d - 1)
                    if i1 < i0:
                        break
                    isl.append(slice(i0, i1 + 1))
                    osl.append(slice(i0 * ss - pp + t, i1 * ss - pp + t + 1, ss))
                if len(osl) < 3:
                    continue
                xs = xc[:, isl[0], isl[1], isl[2], :]
                out[:, osl[0], osl[1], osl[2], :] += torch.matmul(xs, weight[:, :, tz, ty, tx])
    if bias is not None:
        out += bias
    return out.permute(0, 4, 1, 2, 3).contiguous()


@contextlib.contextmanager
def tap_convs():
    """Route torch.nn.functional.conv3d / conv_transpose3d (and so nn.Conv3d / nn.ConvTranspose3d)
    through the tap-GEMM reference inside the block."""
    c, t = F.conv3d, F.conv_transpose3d
    F.conv3d, F.conv_transpose3d = conv3d_taps, conv_transpose3d_taps
    try:
        yield
    finally:
        F.conv3d, F.conv_transpose3d = c, t
