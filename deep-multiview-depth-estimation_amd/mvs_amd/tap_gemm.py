"""Conv3d / ConvTranspose3d with autograd as one rocBLAS GEMM per kernel tap -- the regulariser's
convolutions on the TRAINING path (train.py:97-104: MVSNet.forward under autograd, loss.backward()).

Why: MIOpen has only slow (naive) solvers for the backward passes of the regulariser's 3-D shapes --
the stride-2 convolutions with padding n//2 + 1 (config.py:20) and the full-volume transposed
convolutions -- so one cfg-2 training step took minutes.  Per tap, every convolution pass is a plain
GEMM over channels on channels-last views of the volume (hipBLASLt / rocBLAS through torch.addmm_):

  conv3d forward        y[o] += x[o*s - p + t] @ W_t^T          (o, t per dim; inputs outside = 0)
         d/dx           gx[o*s - p + t] += gy[o] @ W_t
         d/dW           gW_t = sum_o gy[o]^T x[o*s - p + t]
  conv_transpose3d      = the d/dx of the conv3d whose input has the transposed conv's output shape;
                          its d/dx = that conv3d's forward, its d/dW the same sum with x and gy swapped

Layout (no per-tap copies): the conv input is split into its s^3 stride parities and each parity is
stored channels-last on a grid G of the outputs that touch the input (o in [o_lo, o_hi] per dim) plus
(k - 1) // s extra rows: P_a[j] = x[s (o_lo + j) + a - p] (zero outside the input).  Tap t = s d + a
then reads P_a at j = u + d (u = o - o_lo): flattened over (N, G), a CONSTANT row offset
d_z J_y J_x + d_y J_x + d_x, so every tap's operand is a contiguous row range of one matrix and every
pass accumulates in place (beta = 1) into another -- one copy of the volume in and out per pass
instead of one per tap.  Rows whose u falls in the extra rows (or wraps into the next row / sample)
compute garbage that is never read back: the output is taken on [0, O) per dim, and the gradients fed
to the scatters are zero there.

fp32 throughout (gfx950 has no reduced-precision fp32 GEMM mode to fall into); each tap's GEMM sums
over channels, taps are added in a fixed order.  Groups 1, dilation 1, no bias (the reference's
regulariser layers, model.py:76-95).
"""
import torch

_F32 = torch.float32


def _t3(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v, v)


class _Geom:
    """Parity-grid geometry of a conv3d with input extent n, output extent out_n, kernel k, stride s,
    padding p (per dim)."""

    def __init__(self, n, out_n, k, s, p):
        self.n, self.out_n, self.k, self.s, self.p = n, out_n, k, s, p
        self.lo, self.O, self.J = [], [], []
        for d, o, kk, ss, pp in zip(n, out_n, k, s, p):
            lo = max(0, -((kk - 1 - pp) // ss))          # ceil((p - k + 1) / s)
            hi = min(o - 1, (d - 1 + pp) // ss)
            cnt = max(hi - lo + 1, 0)
            self.lo.append(lo)
            self.O.append(cnt)
            self.J.append(cnt + (kk - 1) // ss)
        self.empty = min(self.O) == 0
        self.npar = s[0] * s[1] * s[2]
        Jz, Jy, Jx = self.J
        # per tap (tz, ty, tx): (parity index, row offset)
        self.taps = []
        for tz in range(k[0]):
            for ty in range(k[1]):
                for tx in range(k[2]):
                    a = [t % ss for t, ss in zip((tz, ty, tx), s)]
                    dd = [t // ss for t, ss in zip((tz, ty, tx), s)]
                    pa = (a[0] * s[1] + a[1]) * s[2] + a[2]
                    self.taps.append(((tz, ty, tx), pa, (dd[0] * Jy + dd[1]) * Jx + dd[2]))

    def _par_slices(self, a):
        """(input slices, grid slices) of parity a: the j with 0 <= s (lo + j) + a - p < n."""
        isl, gsl = [], []
        for d, ss, pp, lo, J, aa in zip(self.n, self.s, self.p, self.lo, self.J, a):
            j0 = max(0, -((lo * ss + aa - pp) // ss))       # first j with a nonnegative input index
            j1 = min(J - 1, (d - 1 + pp - aa) // ss - lo)
            if j1 < j0:
                return None
            i0 = ss * (lo + j0) + aa - pp
            isl.append(slice(i0, ss * (lo + j1) + aa - pp + 1, ss))
            gsl.append(slice(j0, j1 + 1))
        return tuple(isl), tuple(gsl)

    def _parities(self):
        s = self.s
        for a0 in range(s[0]):
            for a1 in range(s[1]):
                for a2 in range(s[2]):
                    yield (a0 * s[1] + a1) * s[2] + a2, (a0, a1, a2)

    def to_par(self, xc):
        """channels-last input [N, n..., C] -> [npar, N * J^3, C] parity grids (zeros outside)."""
        N, C = xc.shape[0], xc.shape[-1]
        P = xc.new_zeros((self.npar, N) + tuple(self.J) + (C,))
        for pa, a in self._parities():
            sl = self._par_slices(a)
            if sl is not None:
                P[(pa, slice(None)) + sl[1]] = xc[(slice(None),) + sl[0]]
        return P.view(self.npar, -1, C)

    def from_par(self, P, N, channels_first=False):
        """[npar, N * J^3, C] -> channels-last input-shaped [N, n..., C] (each input voxel lies in one
        parity grid); ``channels_first``: written straight into a contiguous [N, C, n...] tensor instead
        (returned as its channels-last view): the input gradient of an NCDHW input in its own layout, one
        pass, no conversion later."""
        C = P.shape[-1]
        P = P.view((self.npar, N) + tuple(self.J) + (C,))
        if channels_first:
            x = P.new_zeros((N, C) + tuple(self.n)).permute(0, 2, 3, 4, 1)
        else:
            x = P.new_zeros((N,) + tuple(self.n) + (C,))
        for pa, a in self._parities():
            sl = self._par_slices(a)
            if sl is not None:
                x[(slice(None),) + sl[0]] = P[(pa, slice(None)) + sl[1]]
        return x

    def _osl(self):
        return tuple(slice(lo, lo + o) for lo, o in zip(self.lo, self.O))

    def to_grid(self, uc):
        """channels-last output-shaped [N, out_n..., C] -> [N * J^3, C], zero off the valid box."""
        N, C = uc.shape[0], uc.shape[-1]
        G = uc.new_zeros((N,) + tuple(self.J) + (C,))
        G[(slice(None),) + tuple(slice(0, o) for o in self.O)] = uc[(slice(None),) + self._osl()]
        return G.view(-1, C)

    def from_grid(self, G, N):
        """[N * J^3, C] -> channels-last output-shaped [N, out_n..., C] (zeros off the valid box)."""
        C = G.shape[-1]
        G = G.view((N,) + tuple(self.J) + (C,))
        y = G.new_zeros((N,) + tuple(self.out_n) + (C,))
        y[(slice(None),) + self._osl()] = G[(slice(None),) + tuple(slice(0, o) for o in self.O)]
        return y

    # ---- the three passes on parity grids / output grids ----
    def forward(self, P, wt):
        """Y[m] = sum_t P_a(t)[m + off_t] @ wt(t); wt(t) [C_in, C_out]."""
        M = P.shape[1]
        Y = P.new_zeros((M, wt(self.taps[0][0]).shape[1]))
        for t, pa, off in self.taps:
            L = M - off
            Y[:L].addmm_(P[pa, off:off + L], wt(t))
        return Y

    def scatter(self, G, wt, C):
        """gP_a(t)[m + off_t] += G[m] @ wt(t); wt(t) [C_g, C]."""
        M = G.shape[0]
        gP = G.new_zeros((self.npar, M, C))
        for t, pa, off in self.taps:
            L = M - off
            gP[pa, off:off + L].addmm_(G[:L], wt(t))
        return gP

    def weight_grad(self, G, P, out):
        """out(t) = G[:R]^T @ P_a(t)[off_t : off_t + R] for every tap (G zero off the valid box, so
        every tap may use the same R = M - max offset rows).  The sum over ~N J^3 rows is split
        into chunks (a batched GEMM, then a sum over chunks): one GEMM with a K of millions and a
        C_out x C_in output has no parallelism to speak of."""
        M = G.shape[0]
        R = M - max(off for _, _, off in self.taps)
        nch = max(1, min(_KSPLIT, R // 4096))
        rows = R // nch
        Rm = rows * nch
        Cg, Cp = G.shape[1], P.shape[2]
        for t, pa, off in self.taps:
            a = G[:Rm].view(nch, rows, Cg).transpose(1, 2)
            b = P[pa, off:off + Rm].view(nch, rows, Cp)
            v = torch.bmm(a, b).sum(0)
            if Rm < R:
                v = v + torch.matmul(G[Rm:R].t(), P[pa, off + Rm:off + R])
            out(t, v)


_KSPLIT = 256   # row chunks of the weight-gradient GEMMs


def _cl(x):   # [N, C, D, H, W] -> channels-last view [N, D, H, W, C] (to_par / to_grid copy it once)
    return x.permute(0, 2, 3, 4, 1)


def _cf(x):   # channels-last [N, D, H, W, C] -> [N, C, D, H, W] view in channels_last_3d strides
    # (no copy: the next layer's _cl, BatchNorm and the elementwise ops take channels-last as it is)
    return x.permute(0, 4, 1, 2, 3)


class _Conv3dTaps(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, padding, out_size=None):
        s, p, k = _t3(stride), _t3(padding), tuple(w.shape[2:])
        n = tuple(x.shape[2:])
        out_n = (tuple((d + 2 * pp - kk) // ss + 1 for d, pp, kk, ss in zip(n, p, k, s)) if out_size is None
                 else tuple(out_size))
        g = _Geom(n, out_n, k, s, p)
        N = x.shape[0]
        ctx.save_for_backward(x, w)
        ctx.geo = g
        if g.empty:
            return x.new_zeros((N, w.shape[0]) + out_n)
        P = g.to_par(_cl(x))
        ctx.par = P   # the weight gradient's operand: kept instead of formed again from x
        Y = g.forward(P, lambda t: w[(slice(None), slice(None)) + t].t())
        return _cf(g.from_grid(Y, N))

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        g = ctx.geo
        N = x.shape[0]
        gx = gw = None
        if g.empty:
            return (torch.zeros_like(x) if ctx.needs_input_grad[0] else None,
                    torch.zeros_like(w) if ctx.needs_input_grad[1] else None, None, None, None)
        G = g.to_grid(_cl(gy))
        if ctx.needs_input_grad[0]:
            gP = g.scatter(G, lambda t: w[(slice(None), slice(None)) + t], x.shape[1])
            # an NCDHW input (the cost volume) gets its gradient NCDHW: it meets the other readers'
            # gradients (conv_0_0's) and the cost volume's backward in that layout
            gx = _cf(g.from_par(gP, N, channels_first=x.is_contiguous()))
        if ctx.needs_input_grad[1]:
            P = getattr(ctx, "par", None)
            P = g.to_par(_cl(x)) if P is None else P
            gw = torch.zeros_like(w)

            def put(t, v):
                gw[(slice(None), slice(None)) + t] = v
            g.weight_grad(G, P, put)
        ctx.par = None
        return gx, gw, None, None, None


class _ConvTranspose3dTaps(torch.autograd.Function):
    """conv_transpose3d(x) = d/dx of the conv3d g (input extent = this output's, output extent = n)."""

    @staticmethod
    def forward(ctx, x, w, stride, padding, output_padding, out_size=None):
        s, p, op, k = _t3(stride), _t3(padding), _t3(output_padding), tuple(w.shape[2:])
        n = tuple(x.shape[2:])
        out_n = (tuple((d - 1) * ss - 2 * pp + kk + oo for d, ss, pp, kk, oo in zip(n, s, p, k, op))
                 if out_size is None else tuple(out_size))
        g = _Geom(out_n, n, k, s, p)
        N = x.shape[0]
        ctx.save_for_backward(x, w)
        ctx.geo = g
        if g.empty:
            return x.new_zeros((N, w.shape[1]) + out_n)
        G = g.to_grid(_cl(x))
        gP = g.scatter(G, lambda t: w[(slice(None), slice(None)) + t], w.shape[1])
        return _cf(g.from_par(gP, N))

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        g = ctx.geo
        N = x.shape[0]
        gx = gw = None
        if g.empty:
            return (torch.zeros_like(x) if ctx.needs_input_grad[0] else None,
                    torch.zeros_like(w) if ctx.needs_input_grad[1] else None, None, None, None, None)
        P = g.to_par(_cl(gy))
        if ctx.needs_input_grad[0]:
            Y = g.forward(P, lambda t: w[(slice(None), slice(None)) + t].t())
            gx = _cf(g.from_grid(Y, N))
        if ctx.needs_input_grad[1]:
            G = g.to_grid(_cl(x))
            gw = torch.zeros_like(w)

            def put(t, v):
                gw[(slice(None), slice(None)) + t] = v
            g.weight_grad(G, P, put)
        return gx, gw, None, None, None, None


def conv3d_backward(x, w, stride, padding, out_size, gy, need_x=True, need_w=True):
    """(gx, gw) of conv3d_box / conv3d (output u reads inputs u * stride - padding + t, out_size outputs)
    from its input x and output gradient gy: the per-tap-GEMM backward of _Conv3dTaps, for a forward
    computed elsewhere (the HIP region kernels)."""
    s, p, k = _t3(stride), _t3(padding), tuple(w.shape[2:])
    g = _Geom(tuple(x.shape[2:]), tuple(out_size), k, s, p)
    N = x.shape[0]
    if g.empty:
        return (torch.zeros_like(x) if need_x else None), (torch.zeros_like(w) if need_w else None)
    G = g.to_grid(_cl(gy))
    gx = gw = None
    if need_x:
        gP = g.scatter(G, lambda t: w[(slice(None), slice(None)) + t], x.shape[1])
        gx = _cf(g.from_par(gP, N, channels_first=x.is_contiguous()))
    if need_w:
        P = g.to_par(_cl(x))
        gw = torch.zeros_like(w)

        def put(t, v):
            gw[(slice(None), slice(None)) + t] = v
        g.weight_grad(G, P, put)
    return gx, gw


def conv_transpose3d_backward(x, w, stride, crop_lo, out_size, gy, need_x=True, need_w=True):
    """(gx, gw) of conv_transpose3d_box (outputs [crop_lo, crop_lo + out_size) of the unpadded transposed
    conv) from its input x and output gradient gy: _ConvTranspose3dTaps's backward for a forward computed
    elsewhere."""
    s, p, k = _t3(stride), _t3(crop_lo), tuple(w.shape[2:])
    g = _Geom(tuple(out_size), tuple(x.shape[2:]), k, s, p)
    N = x.shape[0]
    if g.empty:
        return (torch.zeros_like(x) if need_x else None), (torch.zeros_like(w) if need_w else None)
    P = g.to_par(_cl(gy))
    gx = gw = None
    if need_x:
        Y = g.forward(P, lambda t: w[(slice(None), slice(None)) + t].t())
        gx = _cf(g.from_grid(Y, N))
    if need_w:
        G = g.to_grid(_cl(x))
        gw = torch.zeros_like(w)

        def put(t, v):
            gw[(slice(None), slice(None)) + t] = v
        g.weight_grad(G, P, put)
    return gx, gw


def conv3d(x, weight, stride=1, padding=0):
    """F.conv3d (groups 1, dilation 1, no bias) through per-tap GEMMs, differentiable."""
    return _Conv3dTaps.apply(x, weight, stride, padding)


def conv_transpose3d(x, weight, stride=1, padding=0, output_padding=0):
    """F.conv_transpose3d (groups 1, dilation 1, no bias) through per-tap GEMMs, differentiable."""
    return _ConvTranspose3dTaps.apply(x, weight, stride, padding, output_padding)


def conv3d_box(x, weight, stride, pad_lo, out_size):
    """Outputs [0, out_size) of a conv3d whose output u reads inputs u * stride - pad_lo + t (pad_lo >= 0:
    zeros before the input; past its end likewise): a box of a padded convolution's output computed as
    a dense tensor (no slice of a larger output)."""
    return _Conv3dTaps.apply(x, weight, stride, pad_lo, out_size)


def conv_transpose3d_box(x, weight, stride, crop_lo, out_size):
    """Outputs [crop_lo, crop_lo + out_size) of the unpadded conv_transpose3d(x, weight, stride) (input i
    reaches outputs i * stride + t), as a dense tensor; outputs past the last input's reach are 0."""
    return _ConvTranspose3dTaps.apply(x, weight, stride, crop_lo, 0, out_size)


class _Conv2dHipTaps(torch.autograd.Function):
    """Conv2d with the HIP forward (ops.conv2d: csrc/conv2d_narrow.hip, exact fp32) and the per-tap-GEMM
    backward of the depth-1 conv3d (the parity grid of x formed in the backward)."""

    @staticmethod
    def forward(ctx, x, w, stride, padding):
        from . import ops
        ctx.save_for_backward(x, w)
        ctx.stride, ctx.padding = stride, padding
        return ops.conv2d(x.contiguous(), w, stride[0])

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        x3, w3 = x.unsqueeze(2), w.unsqueeze(2)
        s, p, k = (1,) + tuple(ctx.stride), (0,) + tuple(ctx.padding), tuple(w3.shape[2:])
        n = tuple(x3.shape[2:])
        out_n = tuple((d + 2 * pp - kk) // ss + 1 for d, pp, kk, ss in zip(n, p, k, s))
        g = _Geom(n, out_n, k, s, p)
        N = x.shape[0]
        G = g.to_grid(_cl(gy.unsqueeze(2)))
        gx = gw = None
        if ctx.needs_input_grad[0]:
            gP = g.scatter(G, lambda t: w3[(slice(None), slice(None)) + t], x.shape[1])
            gx = _cf(g.from_par(gP, N, channels_first=True)).squeeze(2)
        if ctx.needs_input_grad[1]:
            P = g.to_par(_cl(x3))
            gw3 = torch.zeros_like(w3)

            def put(t, v):
                gw3[(slice(None), slice(None)) + t] = v
            g.weight_grad(G, P, put)
            gw = gw3.squeeze(2)
        return gx, gw, None, None


def conv2d(x, weight, stride=1, padding=0):
    """F.conv2d (groups 1, dilation 1, no bias) through the per-tap GEMMs: the conv3d of depth 1."""
    s, p = (stride, stride) if isinstance(stride, int) else tuple(stride), \
        (padding, padding) if isinstance(padding, int) else tuple(padding)
    y = _Conv3dTaps.apply(x.unsqueeze(2), weight.unsqueeze(2), (1,) + tuple(s), (0,) + tuple(p))
    return y.squeeze(2).contiguous()   # NCHW: the BatchNorm2d after it takes MIOpen's NCHW kernels


def conv2d_hip_fwd(x, m):
    """conv2d with the HIP forward kernel and the per-tap-GEMM backward, for a reference layer shape
    (ops.conv2d_supported) on a HIP fp32 NCHW input."""
    return _Conv2dHipTaps.apply(x, m.weight, tuple(m.stride), tuple(m.padding))


def conv2d_applies(m):
    """An nn.Conv2d the per-tap GEMMs run: no bias, groups 1, dilation 1, numeric padding."""
    return (m.bias is None and m.groups == 1 and tuple(m.dilation) == (1, 1)
            and not isinstance(m.padding, str))


def conv_module(m, x):
    """nn.Conv3d / nn.ConvTranspose3d module ``m`` applied through the tap GEMMs."""
    if m.bias is not None or m.groups != 1 or _t3(m.dilation) != (1, 1, 1):
        return m(x)
    if isinstance(m, torch.nn.ConvTranspose3d):
        return conv_transpose3d(x, m.weight, m.stride, m.padding, m.output_padding)
    return conv3d(x, m.weight, m.stride, m.padding)
