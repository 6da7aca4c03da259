"""The regulariser's stride-1 and transposed region convolutions on split-fp16 MFMA
(csrc/conv3d_region_split.hip, ops.conv3d_region_split; model.py:104-120's conv_k_1 / deconv_3_0 /
deconv_2_0 on the eval path) and the bound words that scale their inputs.

Parity: against torch's convolution of the zero-extended tensors in float64 (CPU) -- the same check
test_gpu_parity.py::test_region_conv_matches_torch applies to the fp32-MFMA kernel -- with the error
bounded by the fp32 kernel's own (the split operands carry 22 significant bits; the fp32 accumulation
order is the fp32 kernel's).  Bound words: the kernel raises them to exactly max|y|.
"""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

DEV = torch.device("cuda", 0)


def _bn_params(c, g):
    return (torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.1, torch.randn(c, generator=g) * 0.1)


def _bn_relu(y, sc, sh, mu):
    v = lambda t: t.view(1, -1, 1, 1, 1)
    return torch.relu((y - v(mu)) * v(sc) + v(sh))


def test_split_weight_fragments_host():
    """CPU: mvs_conv3d_region_split_weights lays out hi / lo parts as documented (K-32 blocks; tap pairs
    for c_in = 16), the parts sum to w 2^ew to 2^-22, and tap 27 of the last pair is zero."""
    from mvs_amd.ops import region_split_fragments
    g = torch.Generator().manual_seed(3)
    for cin, cout in ((16, 16), (32, 32), (64, 64), (64, 32), (32, 16)):
        w = torch.randn(27, cout, cin, generator=g) * 0.05
        frag, ew = region_split_fragments(w, torch.device("cpu"))
        kb = 14 if cin == 16 else 27 * cin // 32
        f = frag.view(torch.float16).float().view(kb, cout // 16, 2, 4, 16, 8)   # [kb][nb][part][g][c][j]
        parts = f[:, :, 0] + f[:, :, 1]                                           # [kb][nb][g][c][j]
        # rebuild w[tap][co][ci] * 2^ew from the fragments
        rec = torch.zeros(28 if cin == 16 else 27, cout, cin)
        for k in range(kb):
            for gq in range(4):
                if cin == 16:
                    tap, ci = 2 * k + (gq >> 1), slice(8 * (gq & 1), 8 * (gq & 1) + 8)
                else:
                    tap, c0 = k // (cin // 32), (k % (cin // 32)) * 32 + 8 * gq
                    ci = slice(c0, c0 + 8)
                for nb in range(cout // 16):
                    rec[tap, nb * 16:(nb + 1) * 16, ci] = parts[k, nb, gq]
        ref = w.double() * 2.0 ** ew
        assert w.abs().max().item() * 2.0 ** ew < 2.0 ** 14
        assert (rec[:27].double() - ref).abs().max().item() <= 2.0 ** -21 * ref.abs().max().item()
        if cin == 16:
            assert rec[27].abs().max().item() == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("mode,cin,cout,ncdhw,amp", [(0, 16, 16, False, 1.0), (0, 32, 32, False, 1.0),
                                                    (0, 64, 64, False, 1.0), (2, 64, 32, False, 1.0),
                                                    (2, 32, 16, False, 1.0), (0, 16, 16, True, 1.0),
                                                    (2, 32, 16, True, 1.0), (0, 32, 32, False, 3e3),
                                                    (2, 64, 32, False, 2e-4)])
def test_region_split_conv_matches_torch(mode, cin, cout, ncdhw, amp):
    """conv3d_region_split at forward_live's regions (24 x 20 x 26: odd and even dims, both parities
    of P), channels-last and channels-first, inputs scaled by ``amp`` (the bound words carry the scale):
    max error <= 1e-5 of the output scale against float64 torch and <= 2x the fp32-MFMA kernel's
    (conv3d_region on the same inputs) + 1e-6; the output bound words equal max|y| exactly."""
    from mvs_amd.config import pad_outpad
    from mvs_amd.model import _grow, _tconv_input_region
    from mvs_amd.ops import bound_words, conv3d_region, conv3d_region_split, region_weight
    import torch.nn.functional as F
    n = (24, 20, 26)
    pad, outpad = pad_outpad(*n)
    full = tuple((0, d - 1) for d in n)
    Bx = _tconv_input_region(full, n, pad)
    C2 = _tconv_input_region(Bx, n, pad)
    g = torch.Generator().manual_seed(mode * 100 + cin + cout + int(ncdhw))
    sc, sh, mu = _bn_params(cout, g)
    sh = sh * amp
    mu = mu * amp
    org = lambda r: [lo for lo, _ in r]
    size = lambda r: [hi - lo + 1 for lo, hi in r]
    sl = lambda r: (slice(None), slice(None)) + tuple(slice(lo, hi + 1) for lo, hi in r)
    cl = lambda t: t.permute(0, 2, 3, 4, 1).contiguous()

    def zero_ext(reg, c):
        t = torch.zeros(2, c, *n)
        t[sl(reg)] = torch.relu(torch.randn(2, c, *size(reg), generator=g)) * amp   # post-ReLU activations
        return t

    if mode == 0:      # S1: conv_k_1 on B from halo(B)
        out_reg, in_reg = Bx, _grow(Bx, n, 1)
        x, x2 = zero_ext(in_reg, cin), None
        wt = torch.randn(cout, cin, 3, 3, 3, generator=g) * 0.1
        f = lambda xx, ww: F.conv3d(xx, ww, padding=1)
    else:              # T2: deconv from C2 (+ addend) onto B
        out_reg, in_reg = Bx, C2
        x, x2 = zero_ext(in_reg, cin), zero_ext(in_reg, cin)
        wt = torch.randn(cin, cout, 3, 3, 3, generator=g) * 0.1
        f = lambda xx, ww: F.conv_transpose3d(xx, ww, stride=2, padding=pad, output_padding=outpad)
    xin = x + x2 if x2 is not None else x
    ref64 = _bn_relu(f(xin.double(), wt.double()), sc.double(), sh.double(), mu.double())[sl(out_reg)]
    conv = torch.nn.ConvTranspose3d(cin, cout, 3) if mode == 2 else torch.nn.Conv3d(cin, cout, 3)
    conv.weight.data = wt
    w27 = region_weight(conv).to(DEV)
    bw = bound_words(3, DEV)
    xr = cl(x[sl(in_reg)]).to(DEV)
    x2r = cl(x2[sl(in_reg)]).to(DEV) if x2 is not None else None
    bw[0, 5] = torch.tensor([xr.abs().max().item()], dtype=torch.float32).view(torch.int32).item()
    if x2r is not None:
        bw[1, 0] = torch.tensor([x2r.abs().max().item()], dtype=torch.float32).view(torch.int32).item()
    bn = (sc.to(DEV), sh.to(DEV), mu.to(DEV))
    args = (mode, list(n), org(out_reg), size(out_reg), org(in_reg), size(in_reg), list(pad))
    with torch.no_grad():
        y = conv3d_region_split(xr, x2r, w27, *args, bw[0], None if x2r is None else bw[1], bw[2], *bn,
                                out_ncdhw=ncdhw)
        y32 = conv3d_region(xr, x2r, w27, *args, *bn, out_ncdhw=ncdhw)
        torch.cuda.synchronize()
    ymax = y.abs().max().item()
    got_bound = bw[2].cpu().numpy().view(np.float32).max()
    assert got_bound == ymax, (got_bound, ymax)
    y = (y if ncdhw else y.permute(0, 4, 1, 2, 3)).cpu()
    y32 = (y32 if ncdhw else y32.permute(0, 4, 1, 2, 3)).cpu()
    assert y.shape == ref64.shape
    scale = ref64.abs().max().item()
    err = (y.double() - ref64).abs().max().item()
    err32 = (y32.double() - ref64).abs().max().item()
    assert err <= 1e-5 * scale, (err, scale)
    assert err <= 2 * err32 + 1e-6 * scale, (err, err32, scale)


@pytest.mark.gpu
def test_region_conv_raises_output_bound_words():
    """The fp32-MFMA region kernel (conv3d_region, the S2 conv_k_0 of the split path) raises its
    output's bound words to exactly max|y| -- the scale the split-fp16 conv_k_1 reads."""
    from mvs_amd.config import pad_outpad
    from mvs_amd.model import _grow, _tconv_input_region
    from mvs_amd.ops import bound_words, conv3d_region, region_weight
    n = (24, 20, 26)
    pad, _ = pad_outpad(*n)
    Bx = _tconv_input_region(tuple((0, d - 1) for d in n), n, pad)
    out_reg = _grow(Bx, n, 1)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 32, *n, generator=g).to(DEV)
    conv = torch.nn.Conv3d(32, 32, 3)
    conv.weight.data = torch.randn(32, 32, 3, 3, 3, generator=g) * 0.1
    bw = bound_words(1, DEV)
    with torch.no_grad():
        y = conv3d_region(x, None, region_weight(conv).to(DEV), 1, list(n), [lo for lo, _ in out_reg],
                          [hi - lo + 1 for lo, hi in out_reg], None, None, list(pad), y_bound=bw[0])
        torch.cuda.synchronize()
    words = bw[0].cpu().numpy().view(np.float32)
    assert words.max() == y.abs().max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("cout", [16, 32, 64])
def test_region_split_s2_reads_the_split_volume(cout):
    """conv3d_region_split CONV_S2 (conv_k_0) straight from the split cost volume (its fp16 parts are
    the operands) on forward_live's halo(C2) region: against float64 torch on the volume's fp32 values
    (unsplit_cost_volume) within 1e-5 of the scale and 2x the fp32-MFMA kernel's error (conv3d_region
    reading the same split volume), and with a box of the volume (in_origin / in_size) bit-equal to the
    whole-volume read."""
    from cameras import camera_batch, depth_range
    from mvs_amd import ops
    from mvs_amd.config import pad_outpad
    from mvs_amd.model import _grow, _tconv_input_region
    import torch.nn.functional as F
    B, V, D, h, w = 2, 3, 24, 20, 26
    n = (D, h, w)
    pad, _ = pad_outpad(*n)
    Bx = _tconv_input_region(tuple((0, d - 1) for d in n), n, pad)
    C2 = _tconv_input_region(Bx, n, pad)
    out_reg = _grow(C2, n, 1)
    org, size = [lo for lo, _ in out_reg], [hi - lo + 1 for lo, hi in out_reg]
    K, R, T = camera_batch(B, V, h, w)
    d_min, d_int = depth_range(B, d_int=200.0 / D)
    g = torch.Generator().manual_seed(cout)
    feat = torch.randn(B * V, 32, h, w, generator=g).to(DEV)
    conv = torch.nn.Conv3d(32, cout, 3)
    conv.weight.data = torch.randn(cout, 32, 3, 3, 3, generator=g) * 0.1
    sc, sh, mu = _bn_params(cout, g)
    bn = (sc.to(DEV), sh.to(DEV), mu.to(DEV))
    w27 = ops.region_weight(conv).to(DEV)
    with torch.no_grad():
        scv, am = ops.cost_volume_c4_split(feat, K, R, T, d_min, d_int, B, V, 0, D, 25.0)
        xv = ops.unsplit_cost_volume(scv, am)                      # [B, 8, D, h, w, 4] fp32 values
        xv = xv.permute(0, 1, 5, 2, 3, 4).reshape(B, 32, *n).cpu()
        bw = ops.bound_words(1, DEV)
        y = ops.conv3d_region_split(scv, None, w27, ops.CONV_S2, list(n), org, size, None, None, list(pad), am, None,
                                    bw[0], *bn)
        y32 = ops.conv3d_region(scv, None, w27, ops.CONV_S2, list(n), org, size, None, None, list(pad), *bn,
                                in_c4=True, absmax=am)
        # the box of the volume the windows read (what the opt-in fused head stores)
        lo = [max(2 * a - p, 0) for (a, _), p in zip(out_reg, pad)]
        hi = [min(2 * b - p + 2, d - 1) + 1 for (_, b), p, d in zip(out_reg, pad, n)]
        box = scv[:, :, lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]].contiguous()
        yb = ops.conv3d_region_split(box, None, w27, ops.CONV_S2, list(n), org, size, lo,
                                     [b - a for a, b in zip(lo, hi)], list(pad), am, None, None, *bn)
        torch.cuda.synchronize()
    sl = (slice(None), slice(None)) + tuple(slice(a, b + 1) for a, b in out_reg)
    ref64 = _bn_relu(F.conv3d(xv.double(), conv.weight.double(), stride=2, padding=pad), sc.double(), sh.double(),
                     mu.double())[sl]
    yc, y32c = y.permute(0, 4, 1, 2, 3).cpu(), y32.permute(0, 4, 1, 2, 3).cpu()
    scale = ref64.abs().max().item()
    err = (yc.double() - ref64).abs().max().item()
    err32 = (y32c.double() - ref64).abs().max().item()
    assert err <= 1e-5 * scale, (err, scale)
    assert err <= 2 * err32 + 1e-6 * scale, (err, err32)
    assert bw[0].cpu().numpy().view(np.float32).max() == y.abs().max().item()
    assert torch.equal(yb, y)


@pytest.mark.gpu
@pytest.mark.parametrize("c,ncdhw,shape", [(16, False, (24, 20, 26)), (16, True, (13, 11, 37)), (32, False, (24, 20, 26)),
                                           (32, False, (9, 7, 17)), (32, True, (11, 5, 50))])
def test_region_split_s1_lds_equals_per_lane(c, ncdhw, shape):
    """The LDS-staged stride-1 kernel (the default for the 16- and 32-channel conv_k_1) is bit-identical to the per-lane-operand
    kernel (MVS_CONV_PER_LANE) -- same products in the same order -- on regions that are not multiples
    of its 16 x 4 x TZ tile, with and without BN, and raises the same bound words."""
    from mvs_amd.model import _grow, _tconv_input_region
    from mvs_amd.config import pad_outpad
    from mvs_amd.ops import CONV_S1, bound_words, conv3d_region_split, region_weight
    n = shape
    pad, _ = pad_outpad(*n)
    Bx = _tconv_input_region(tuple((0, d - 1) for d in n), n, pad)
    out_reg, in_reg = Bx, _grow(Bx, n, 1)
    org = lambda r: [lo for lo, _ in r]
    size = lambda r: [hi - lo + 1 for lo, hi in r]
    g = torch.Generator().manual_seed(c + sum(n))
    x = (torch.relu(torch.randn(2, *size(in_reg), c, generator=g)) * 3).to(DEV)
    conv = torch.nn.Conv3d(c, c, 3)
    conv.weight.data = torch.randn(c, c, 3, 3, 3, generator=g) * 0.1
    w27 = region_weight(conv).to(DEV)
    bw = bound_words(3, DEV)
    bw[0, 7] = torch.tensor([x.abs().max().item()], dtype=torch.float32).view(torch.int32).item()
    args = (CONV_S1, list(n), org(out_reg), size(out_reg), org(in_reg), size(in_reg), None)
    for bn in ((None, None, None), tuple(t.to(DEV) for t in _bn_params(c, g))):
        bw[1:].zero_()
        with torch.no_grad():
            a = conv3d_region_split(x, None, w27, *args, bw[0], None, bw[1], *bn, out_ncdhw=ncdhw)
            b = conv3d_region_split(x, None, w27, *args, bw[0], None, bw[2], *bn, out_ncdhw=ncdhw, per_lane=True)
            torch.cuda.synchronize()
        assert torch.equal(a, b), (a - b).abs().max().item()
        assert bw[1].max().item() == bw[2].max().item()


@pytest.mark.gpu
def test_region_split_output_addend():
    """y_addend (deconv_3_0's `+ y2`, model.py:119, formed in its epilogue) adds after BN + ReLU: bit-equal
    to the output plus the addend, and the bound words bound the sum."""
    from mvs_amd.model import _tconv_input_region
    from mvs_amd.config import pad_outpad
    from mvs_amd.ops import CONV_T2, bound_words, conv3d_region_split, region_weight
    n = (24, 20, 26)
    pad, _ = pad_outpad(*n)
    Bx = _tconv_input_region(tuple((0, d - 1) for d in n), n, pad)
    C2 = _tconv_input_region(Bx, n, pad)
    org = lambda r: [lo for lo, _ in r]
    size = lambda r: [hi - lo + 1 for lo, hi in r]
    g = torch.Generator().manual_seed(21)
    x = torch.relu(torch.randn(2, *size(C2), 64, generator=g)).to(DEV)
    conv = torch.nn.ConvTranspose3d(64, 32, 3)
    conv.weight.data = torch.randn(64, 32, 3, 3, 3, generator=g) * 0.1
    w27 = region_weight(conv).to(DEV)
    bn = tuple(t.to(DEV) for t in _bn_params(32, g))
    bw = bound_words(3, DEV)
    bw[0, 0] = torch.tensor([x.abs().max().item()], dtype=torch.float32).view(torch.int32).item()
    add = torch.relu(torch.randn(2, *size(Bx), 32, generator=g)).to(DEV)
    args = (CONV_T2, list(n), org(Bx), size(Bx), org(C2), size(C2), list(pad))
    with torch.no_grad():
        y = conv3d_region_split(x, None, w27, *args, bw[0], None, bw[1], *bn)
        ys = conv3d_region_split(x, None, w27, *args, bw[0], None, bw[2], *bn, y_addend=add)
        torch.cuda.synchronize()
    assert torch.equal(ys, y + add)
    assert bw[2].cpu().numpy().view(np.float32).max() == ys.abs().max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("mode,cin,cout,ncdhw", [(0, 16, 16, True), (0, 32, 32, False), (0, 64, 64, False),
                                                 (2, 64, 32, False), (2, 32, 16, True), (1, 32, 16, False),
                                                 (1, 32, 64, False)])
def test_region_split_sums_and_store_box(mode, cin, cout, ncdhw):
    """Train-mode BatchNorm's batch sums formed in the split kernels' epilogues (conv3d_region_split_sums,
    DESIGN.md §5b): the per-channel float64 sum / sum of squares over the whole output region equal
    channel_stats of the un-boxed output (1e-12 relative), the stored box is bit-equal to that output's
    crop, and two launches give bit-identical sums (slot-owned partials, fixed-order total).  S1 on
    R1 -> stored M (LDS kernel for 16 / 32 channels, per-lane for 64), T2 full volume -> stored M, S2
    from the split cost volume on R2 (stored whole)."""
    from cameras import camera_batch, depth_range
    from mvs_amd import ops
    from mvs_amd.config import pad_outpad
    from mvs_amd.model import _grow, _tconv_input_region
    B, D, h, w = 2, 24, 20, 26
    n = (D, h, w)
    pad, _ = pad_outpad(*n)
    full = tuple((0, d - 1) for d in n)
    M = _tconv_input_region(full, n, pad)
    R1, R2 = _grow(M, n, 1), _grow(M, n, 2)
    org = lambda r: [lo for lo, _ in r]
    size = lambda r: [hi - lo + 1 for lo, hi in r]
    g = torch.Generator().manual_seed(mode * 1000 + cin + cout)
    conv = torch.nn.ConvTranspose3d(cin, cout, 3) if mode == 2 else torch.nn.Conv3d(cin, cout, 3)
    conv.weight.data = torch.randn(*conv.weight.shape, generator=g) * 0.1
    w27 = ops.region_weight(conv).to(DEV)
    bw = ops.bound_words(1, DEV)
    with torch.no_grad():
        if mode == 1:   # S2: conv_k_0 from the split cost volume on R2
            K, R, T = camera_batch(B, 3, h, w)
            d_min, d_int = depth_range(B, d_int=200.0 / D)
            feat = torch.randn(B * 3, 32, h, w, generator=g).to(DEV)
            x, xb = ops.cost_volume_c4_split(feat, K, R, T, d_min, d_int, B, 3, 0, D, 25.0)
            geo = (ops.CONV_S2, list(n), org(R2), size(R2), None, None, list(pad))
            box = R2
        else:
            in_reg = R2 if mode == 0 else M
            x = torch.relu(torch.randn(B, *size(in_reg), cin, generator=g)).to(DEV)
            xb = bw[0]
            xb[0] = x.abs().max().view(torch.int32)
            out_reg = R1 if mode == 0 else full
            geo = (mode, list(n), org(out_reg), size(out_reg), org(in_reg), size(in_reg),
                   None if mode == 0 else list(pad))
            box = M
        out_reg = [(o, o + s - 1) for o, s in zip(geo[2], geo[3])]
        y_full = ops.conv3d_region_split(x, None, w27, *geo, xb, None, None, out_ncdhw=ncdhw)
        r1, r2 = ops.channel_stats(y_full, not ncdhw)
        ys, s1, s2 = ops.conv3d_region_split_sums(x, None, w27, *geo, xb, out_ncdhw=ncdhw, store_origin=org(box),
                                                  store_size=size(box))
        _, t1, t2 = ops.conv3d_region_split_sums(x, None, w27, *geo, xb, out_ncdhw=ncdhw, store_origin=org(box),
                                                 store_size=size(box))
        torch.cuda.synchronize()
    crop = [slice(lo - olo, hi - olo + 1) for (olo, _), (lo, hi) in zip(out_reg, box)]
    want = y_full[:, :, crop[0], crop[1], crop[2]] if ncdhw else y_full[:, crop[0], crop[1], crop[2], :]
    assert torch.equal(ys, want.contiguous())
    torch.testing.assert_close(s1, r1, rtol=1e-12, atol=1e-9)
    torch.testing.assert_close(s2, r2, rtol=1e-12, atol=1e-9)
    assert torch.equal(s1, t1) and torch.equal(s2, t2)


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,ncdhw,n", [(64, 32, False, (24, 20, 26)), (32, 16, True, (24, 20, 26)),
                                              (64, 32, False, (13, 9, 37)), (32, 16, False, (20, 17, 70))])
def test_region_split_t2_lds_kernel_is_bit_equal(cin, cout, ncdhw, n, monkeypatch):
    """The LDS-staged transposed kernel (train mode's full-volume deconv_3_0 / deconv_2_0;
    MVS_T2_LDS=2 forces it) against the per-lane kernel on the full output volume from the middle-half
    input region: bit-equal outputs (same products, same K order) with BN epilogue and an output
    addend, bit-equal stored boxes, equal bound words, and the fused sums within 1e-12 (the workgroups,
    and so the partial sums, are partitioned differently)."""
    from mvs_amd import ops
    from mvs_amd.config import pad_outpad
    from mvs_amd.model import _tconv_input_region
    pad, _ = pad_outpad(*n)
    full = tuple((0, d - 1) for d in n)
    M = _tconv_input_region(full, n, pad)
    org = lambda r: [lo for lo, _ in r]
    size = lambda r: [hi - lo + 1 for lo, hi in r]
    g = torch.Generator().manual_seed(cin + sum(n))
    conv = torch.nn.ConvTranspose3d(cin, cout, 3)
    conv.weight.data = torch.randn(*conv.weight.shape, generator=g) * 0.1
    w27 = ops.region_weight(conv).to(DEV)
    x = torch.relu(torch.randn(2, *size(M), cin, generator=g)).to(DEV)
    bw = ops.bound_words(3, DEV)
    bw[0, 0] = x.abs().max().view(torch.int32)
    sc, sh, mu = (t.to(DEV) for t in _bn_params(cout, g))
    geo = (ops.CONV_T2, list(n), [0, 0, 0], list(n), org(M), size(M), list(pad))
    shape = (2, cout) + tuple(n) if ncdhw else (2,) + tuple(n) + (cout,)
    add = torch.randn(shape, generator=g).to(DEV)
    with torch.no_grad():
        monkeypatch.setenv("MVS_T2_LDS", "2")
        y = ops.conv3d_region_split(x, None, w27, *geo, bw[0], None, bw[1], sc, sh, mu, out_ncdhw=ncdhw, y_addend=add)
        ys, s1, s2 = ops.conv3d_region_split_sums(x, None, w27, *geo, bw[0], out_ncdhw=ncdhw, store_origin=org(M),
                                                  store_size=size(M))
        monkeypatch.setenv("MVS_T2_LDS", "0")
        ref = ops.conv3d_region_split(x, None, w27, *geo, bw[0], None, bw[2], sc, sh, mu, out_ncdhw=ncdhw,
                                      y_addend=add)
        rs, r1, r2 = ops.conv3d_region_split_sums(x, None, w27, *geo, bw[0], out_ncdhw=ncdhw, store_origin=org(M),
                                                  store_size=size(M))
        torch.cuda.synchronize()
    assert torch.equal(y, ref)
    assert torch.equal(bw[1].max(), bw[2].max())
    assert torch.equal(ys, rs)
    torch.testing.assert_close(s1, r1, rtol=1e-12, atol=1e-9)
    torch.testing.assert_close(s2, r2, rtol=1e-12, atol=1e-9)


@pytest.mark.gpu
def test_region_split_s2_multi_equals_three_launches():
    """Train mode's conv_1_0 / conv_2_0 / conv_3_0 in one launch (ops.conv_s2_split_multi_sums, c_out
    16 + 32 + 64 over the same region of the split cost volume) against three conv3d_region_split_sums
    launches: the same outputs (one weight exponent for the three weights: the products are the same up
    to a power of two) and the same batch sums."""
    from cameras import camera_batch, depth_range
    from mvs_amd import ops
    from mvs_amd.config import pad_outpad
    from mvs_amd.model import _grow, _tconv_input_region
    B, D, h, w = 2, 24, 20, 26
    n = (D, h, w)
    pad, _ = pad_outpad(*n)
    M = _tconv_input_region(tuple((0, d - 1) for d in n), n, pad)
    R2 = _grow(M, n, 2)
    org, size = [lo for lo, _ in R2], [hi - lo + 1 for lo, hi in R2]
    g = torch.Generator().manual_seed(17)
    K, R, T = camera_batch(B, 3, h, w)
    d_min, d_int = depth_range(B, d_int=200.0 / D)
    feat = torch.randn(B * 3, 32, h, w, generator=g).to(DEV)
    ws = []
    for c, scale in ((16, 0.1), (32, 0.03), (64, 0.2)):   # different magnitudes: one shared exponent
        conv = torch.nn.Conv3d(32, c, 3)
        conv.weight.data = torch.randn(c, 32, 3, 3, 3, generator=g) * scale
        ws.append(ops.region_weight(conv).to(DEV))
    with torch.no_grad():
        scv, am = ops.cost_volume_c4_split(feat, K, R, T, d_min, d_int, B, 3, 0, D, 25.0)
        multi = ops.conv_s2_split_multi_sums(scv, ws, list(n), org, size, list(pad), am)
        for (y, s1, s2), wk in zip(multi, ws):
            ry, r1, r2 = ops.conv3d_region_split_sums(scv, None, wk, ops.CONV_S2, list(n), org, size, None, None,
                                                      list(pad), am)
            torch.testing.assert_close(y, ry, rtol=1e-6, atol=1e-6 * ry.abs().max().item())
            torch.testing.assert_close(s1, r1, rtol=1e-9, atol=1e-6)
            torch.testing.assert_close(s2, r2, rtol=1e-9, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,two", [(64, 32, False), (32, 16, True)])
def test_region_split_t2_folded_input_bn(cin, cout, two, monkeypatch):
    """Train mode's BN + ReLU folded into the LDS transposed kernel's staging (x_bn / x2_bn): equal to
    the same kernel on the explicitly normalised (and summed) input within fp32-level error -- the input
    scale then comes from a bound of relu(BN(.)) over the raw tensors' bound words, a few bits coarser than
    the normalised tensor's own -- with the same batch sums."""
    from mvs_amd import ops
    from mvs_amd.config import pad_outpad
    from mvs_amd.model import _tconv_input_region
    n = (24, 20, 26)
    pad, _ = pad_outpad(*n)
    full = tuple((0, d - 1) for d in n)
    M = _tconv_input_region(full, n, pad)
    org = lambda r: [lo for lo, _ in r]
    size = lambda r: [hi - lo + 1 for lo, hi in r]
    g = torch.Generator().manual_seed(cin * 3 + int(two))
    conv = torch.nn.ConvTranspose3d(cin, cout, 3)
    conv.weight.data = torch.randn(*conv.weight.shape, generator=g) * 0.1
    w27 = ops.region_weight(conv).to(DEV)
    raw = [torch.randn(2, *size(M), cin, generator=g).to(DEV) for _ in range(2 if two else 1)]
    bns = [tuple(t.to(DEV) for t in _bn_params(cin, g)) for _ in raw]
    bw = ops.bound_words(4, DEV)
    for k, r in enumerate(raw):
        bw[k, 0] = r.abs().max().view(torch.int32)
    norm = sum(torch.relu((r - p[2]) * p[0] + p[1]) for r, p in zip(raw, bns))
    bw[2, 0] = norm.abs().max().view(torch.int32)
    geo = (ops.CONV_T2, list(n), [0, 0, 0], list(n), org(M), size(M), list(pad))
    with torch.no_grad():
        monkeypatch.setenv("MVS_T2_LDS", "2")
        ref, r1, r2 = ops.conv3d_region_split_sums(norm.contiguous(), None, w27, *geo, bw[2], store_origin=org(M),
                                                   store_size=size(M))
        got, s1, s2 = ops.conv3d_region_split_sums(raw[0], raw[1] if two else None, w27, *geo, bw[0],
                                                   x2_bound=bw[1] if two else None, store_origin=org(M),
                                                   store_size=size(M), x_bn=bns[0], x2_bn=bns[1] if two else None)
        torch.cuda.synchronize()
    scale = ref.abs().max().item()
    assert (got - ref).abs().max().item() <= 2e-6 * scale
    torch.testing.assert_close(s1, r1, rtol=1e-5, atol=1e-5 * scale)
    torch.testing.assert_close(s2, r2, rtol=1e-5, atol=1e-5 * scale * scale)


@pytest.mark.gpu
@pytest.mark.parametrize("c", [16, 32])
def test_region_split_s1_folded_input_bn(c):
    """Train mode's conv_k_0 BN + ReLU folded into conv_k_1's LDS staging (x_bn on CONV_S1 16 / 32
    channels): equal to the same kernel on the explicitly normalised input within fp32-level error, the
    zero padding outside the volume left zero (not relu(BN(0))), and the same batch sums."""
    from mvs_amd import ops
    from mvs_amd.config import pad_outpad
    from mvs_amd.model import _grow, _tconv_input_region
    n = (24, 20, 26)
    pad, _ = pad_outpad(*n)
    M = _tconv_input_region(tuple((0, d - 1) for d in n), n, pad)
    R1, R2 = _grow(M, n, 1), _grow(M, n, 2)
    org = lambda r: [lo for lo, _ in r]
    size = lambda r: [hi - lo + 1 for lo, hi in r]
    g = torch.Generator().manual_seed(c + 5)
    conv = torch.nn.Conv3d(c, c, 3)
    conv.weight.data = torch.randn(c, c, 3, 3, 3, generator=g) * 0.1
    w27 = ops.region_weight(conv).to(DEV)
    raw = torch.randn(2, *size(R2), c, generator=g).to(DEV)
    p = tuple(t.to(DEV) for t in _bn_params(c, g))
    norm = torch.relu((raw - p[2]) * p[0] + p[1]).contiguous()
    bw = ops.bound_words(2, DEV)
    bw[0, 0] = raw.abs().max().view(torch.int32)
    bw[1, 0] = norm.abs().max().view(torch.int32)
    geo = (ops.CONV_S1, list(n), org(R1), size(R1), org(R2), size(R2), None)
    with torch.no_grad():
        ref, r1, r2 = ops.conv3d_region_split_sums(norm, None, w27, *geo, bw[1], store_origin=org(M),
                                                   store_size=size(M))
        got, s1, s2 = ops.conv3d_region_split_sums(raw, None, w27, *geo, bw[0], store_origin=org(M),
                                                   store_size=size(M), x_bn=p)
        torch.cuda.synchronize()
    scale = ref.abs().max().item()
    assert (got - ref).abs().max().item() <= 2e-6 * scale
    torch.testing.assert_close(s1, r1, rtol=1e-5, atol=1e-5 * scale)
    torch.testing.assert_close(s2, r2, rtol=1e-5, atol=1e-5 * scale * scale)


@pytest.mark.gpu
def test_conv_out_folded_input_bn():
    """Train mode's conv_out input relu(BN_0(deconv_1_0)) + relu(BN_0'(conv_0_0)) formed in conv_out's
    staging (conv3d_k3 x2 / in_bn) against the bn_relu_ pass followed by conv3d_k3 (model.py:121-123):
    equal within fp32 rounding, including the volume border (the zero padding stays zero)."""
    from mvs_amd import ops
    g = torch.Generator().manual_seed(21)
    shape = (2, 8, 13, 18, 37)
    z = torch.randn(shape, generator=g).to(DEV)
    y0 = torch.randn(shape, generator=g).to(DEV)
    pa = [t.to(DEV) for t in _bn_params(8, g)]
    pb = [t.to(DEV) for t in _bn_params(8, g)]
    w = (torch.randn(1, 8, 3, 3, 3, generator=g) * 0.2).to(DEV)
    with torch.no_grad():
        ref = ops.conv3d_k3(ops.bn_relu_(z.clone(), False, *pa, r=y0, r_bn=pb), w)
        got = ops.conv3d_k3(z, w, x2=y0, in_bn=torch.stack(pa + pb))
    torch.testing.assert_close(got, ref, rtol=1e-6, atol=1e-6 * ref.abs().max().item())
