"""Split-fp16 conv_0_0 (csrc/conv3d_split.hip, mvs_conv3d_k3_split_fwd / ops.conv3d_k3_split).

CPU (no GPU): the host-side weight split (mvs_conv3d_split_weights) -- fragment layout against the
16x16x32 MFMA operand map, hi + lo within 2^-22 of the scaled weight, the exponent rule.

GPU: the kernel against float64 (torch CPU) on the same volumes, and against the exact-fp32 kernel
(conv3d_k3) and torch's fp32 Conv3d (MIOpen): the split arithmetic must carry fp32-level error --
max error <= 1e-5 of the output scale and no more than 1.5x the larger of the two fp32 kernels'
own errors (+ 1e-7 of scale).  Cases: ragged x / y tiles and depth chunks, with and without the fused
eval BN + ReLU, volumes from the fused cost-volume kernel with their bound words, and synthetic
volumes far outside fp16's range (values to 1e9, the bound scales them) and far below it (1e-6).
"""
import ctypes

import numpy as np
import pytest
import torch

from mvs_amd import _lib


def _split_host(w):
    lib = _lib.load()
    w = w.to(torch.float32).contiguous()
    frag = torch.empty((27 * 64 * 8,), dtype=torch.int16)
    e = ctypes.c_int(0)
    st = lib.mvs_conv3d_split_weights(_lib.ptr(w), _lib.ptr(frag), ctypes.byref(e))
    return st, frag.view(torch.float16).reshape(27, 64, 8).to(torch.float64), e.value


def test_split_weights_layout_and_accuracy():
    g = torch.Generator().manual_seed(5)
    w = torch.randn(8, 32, 3, 3, 3, generator=g) * 0.05
    st, frag, ew = _split_host(w)
    assert st == 0
    m = w.abs().max().item()
    assert m * 2.0 ** ew < 2 ** 14 <= 2 * m * 2.0 ** ew          # the largest power of two that fits
    ws = w.double() * 2.0 ** ew
    lane = torch.arange(64)
    col, grp = lane & 15, lane >> 4
    for tap in (0, 4, 13, 26):
        kz, ky, kx = tap // 9, (tap // 3) % 3, tap % 3
        hi = torch.zeros(8, 32, dtype=torch.float64)
        lo = torch.zeros(8, 32, dtype=torch.float64)
        for l in range(64):
            for j in range(8):
                c, ci = int(col[l]), 8 * int(grp[l]) + j
                (hi if c < 8 else lo)[c & 7, ci] = frag[tap, l, j]
        ref = ws[:, :, kz, ky, kx]
        assert torch.equal(hi, ref.to(torch.float16).double())            # hi = nearest fp16
        assert (hi + lo - ref).abs().max() <= 2.0 ** -22 * ref.abs().max() + 2.0 ** -24


def test_split_weights_rejects_non_finite():
    w = torch.zeros(8, 32, 3, 3, 3)
    st, _, ew = _split_host(w)
    assert st == 0 and ew == 0
    w[1, 2, 0, 1, 2] = float("nan")
    assert _split_host(w)[0] == -1   # MVS_ERR_INVALID_ARGUMENT


DEV = torch.device("cuda:0")


def _bound_words(x_ncdhw):
    """int32[8] bound words for a synthetic volume: sqrt(max|x|) rounded up, in word 3."""
    b = np.float32(np.sqrt(float(x_ncdhw.abs().max())) * (1 + 1e-6))
    words = torch.zeros(8, dtype=torch.int32)
    words[3] = int(np.frombuffer(b.tobytes(), dtype=np.int32)[0])
    return words


def _to_c4(x):
    b, c, d, h, w = x.shape
    return x.reshape(b, c // 4, 4, d, h, w).permute(0, 1, 3, 4, 5, 2).contiguous()


def _check(x, wt, bn, absmax, label):
    from mvs_amd.ops import conv3d_k3, conv3d_k3_split
    ref64 = torch.nn.functional.conv3d(x.double(), wt.double(), padding=1)
    if bn is not None:
        sc, sh, mu = (t.double()[:, None, None, None] for t in bn)
        ref64 = torch.clamp((ref64 - mu) * sc + sh, min=0.0)
    bdev = [t.to(DEV) for t in bn] if bn is not None else []
    with torch.no_grad():
        xc = _to_c4(x).to(DEV)
        y = conv3d_k3_split(xc, None if absmax is None else absmax.to(DEV), wt.to(DEV), *bdev).cpu()
        y32 = conv3d_k3(xc, wt.to(DEV), *bdev, in_c4=True).cpu()
        yt = torch.nn.functional.conv3d(x.to(DEV), wt.to(DEV), padding=1)
        if bn is not None:
            sc, sh, mu = (t.to(DEV)[:, None, None, None] for t in bn)
            yt = torch.clamp((yt - mu) * sc + sh, min=0.0)
        yt = yt.cpu()
    scale = ref64.abs().max().item()
    err = (y.double() - ref64).abs().max().item()
    err32 = (y32.double() - ref64).abs().max().item()
    errt = (yt.double() - ref64).abs().max().item()
    print("%s: split %.3g, fp32 kernel %.3g, MIOpen %.3g (scale %.3g)" % (label, err, err32, errt, scale))
    assert torch.isfinite(y).all()
    assert err <= 1e-5 * scale, (label, err, scale)
    assert err <= 1.5 * max(err32, errt) + 1e-7 * scale, (label, err, err32, errt)
    return err, err32, errt


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(1, 9, 20, 33), (2, 37, 17, 48), (1, 64, 24, 160)])
@pytest.mark.parametrize("bn", [False, True])
def test_split_conv_synthetic(shape, bn):
    """Ragged tiles (W not a multiple of 16 or 4, H of 8, D of 4 / 32), BN epilogue on / off, a
    cost-volume-like non-negative input with its bound words."""
    b, d, h, w = shape
    g = torch.Generator().manual_seed(sum(shape) + bn)
    x = torch.randn(b, 32, d, h, w, generator=g).square()
    wt = torch.randn(8, 32, 3, 3, 3, generator=g) * 0.05
    p = (torch.rand(8, generator=g) + 0.5, torch.randn(8, generator=g), torch.randn(8, generator=g) * 0.1) if bn else None
    _check(x, wt, p, _bound_words(x), "synthetic %s bn=%s" % (shape, bn))


@pytest.mark.gpu
@pytest.mark.parametrize("mag", [1e-6, 1.0, 1e9])
def test_split_conv_magnitudes(mag):
    """Values far below fp16's normal range and far above its maximum: the bound's power-of-two scale
    keeps the split exact-ish (unscaled, 1e9 would overflow fp16)."""
    g = torch.Generator().manual_seed(int(np.log10(mag)) + 40)
    x = torch.rand(1, 32, 10, 16, 40, generator=g) * mag
    wt = torch.randn(8, 32, 3, 3, 3, generator=g) * 3.0
    _check(x, wt, None, _bound_words(x), "magnitude %g" % mag)


@pytest.mark.gpu
@pytest.mark.parametrize("small", [1e-6, 1e-8])
def test_split_conv_dynamic_range(small):
    """One volume, two dynamic ranges: depth planes 0-5 at scale 1, planes 6-11 at `small` x that
    (the split's power-of-two scale is set by the volume's bound, so the small region's values sit
    near fp16's subnormal range).  Per output region, split vs float64, exact fp32 (conv3d_k3) and
    MIOpen vs float64.  The split's element contract:

        |x - (hi + lo) 2^-e| <= 2^-22 |x| + 2^-25 2^-e,   2^-e <= B^2 2^-12   (B = the bound word)

    -- fp32-level relative error down to ~1e-5 of the volume's bound, an ABSOLUTE floor of
    B^2 2^-37 (7e-12 B^2) below.  Asserted: the large region at fp32 level (as every other test
    here); in the small region the error within the contract's propagated bound
    sum_taps |w| (2^-22 max|x| + 2^-37 B^2) + the fp32 kernels' own error, and the measured
    relative errors recorded."""
    from conftest import record_parity
    from mvs_amd.ops import conv3d_k3, conv3d_k3_split
    g = torch.Generator().manual_seed(71)
    x = torch.rand(1, 32, 12, 16, 40, generator=g)
    x[:, :, 6:] *= small
    wt = torch.randn(8, 32, 3, 3, 3, generator=g) * 0.05
    words = _bound_words(x)
    bound2 = float(np.frombuffer(np.int32(words[3].item()).tobytes(), dtype=np.float32)[0]) ** 2
    ref64 = torch.nn.functional.conv3d(x.double(), wt.double(), padding=1)
    with torch.no_grad():
        xc = _to_c4(x).to(DEV)
        y = conv3d_k3_split(xc, words.to(DEV), wt.to(DEV)).cpu().double()
        y32 = conv3d_k3(xc, wt.to(DEV), in_c4=True).cpu().double()
        yt = torch.nn.functional.conv3d(x.to(DEV), wt.to(DEV), padding=1).cpu().double()
    big, sm = (slice(None), slice(None), slice(0, 5)), (slice(None), slice(None), slice(7, 12))
    out = {}
    for name, r in (("large", big), ("small", sm)):
        scale = ref64[r].abs().max().item()
        e_s, e_32, e_t = ((v[r] - ref64[r]).abs().max().item() for v in (y, y32, yt))
        out[name] = dict(scale=scale, split_rel=e_s / scale, fp32_kernel_rel=e_32 / scale, miopen_rel=e_t / scale)
        print("%s region (x %g): split %.3g, fp32 kernel %.3g, MIOpen %.3g relative to %.3g" % (
            name, 1.0 if name == "large" else small, e_s / scale, e_32 / scale, e_t / scale, scale))
        if name == "large":
            assert e_s <= 1e-5 * scale and e_s <= 1.5 * max(e_32, e_t) + 1e-7 * scale, out[name]
        else:
            sw = wt.double().abs().sum((1, 2, 3, 4)).max().item()
            contract = sw * (2.0 ** -22 * x[:, :, 6:].abs().max().item() + 2.0 ** -37 * bound2)
            out[name]["contract_bound"] = contract / scale
            assert e_s <= contract + 2 * max(e_32, e_t), out[name]
    record_parity("split_dynamic_range_%g" % small, **out)


@pytest.mark.gpu
def test_split_conv_unscaled_small_values():
    """absmax = None: unscaled (values < 2^15 by contract)."""
    g = torch.Generator().manual_seed(3)
    x = torch.rand(1, 32, 8, 12, 20, generator=g) * 100.0
    wt = torch.randn(8, 32, 3, 3, 3, generator=g) * 0.05
    _check(x, wt, None, None, "unscaled")


@pytest.mark.gpu
def test_split_conv_on_fused_cost_volume():
    """The production pairing: cost_volume_c4_absmax (bound words from the prologue's max|feat|)
    feeding conv3d_k3_split, B=2 V=3 with distinct depth ranges, against float64 of that volume;
    every volume element within the bound."""
    from cameras import camera_batch, depth_range, features
    from mvs_amd import ops
    B, V, C, h, w, D = 2, 3, 32, 40, 52, 12
    K, R, T = camera_batch(B, V, h, w)
    d_min, d_int = depth_range(B, d_int=4.0, distinct=True)
    feat = features(B * V, C, h, w, seed=11) * 7.0
    with torch.no_grad():
        cv, absmax = ops.cost_volume_c4_absmax(feat.to(DEV), K, R, T, d_min, d_int, B, V, 0, D, 25.0)
    words = absmax.cpu()
    bound = np.frombuffer(words.numpy().astype(np.int32).tobytes(), dtype=np.float32).max()
    assert bound == np.float32(feat.abs().max().item())          # exactly max|feat|
    x = cv.cpu().permute(0, 1, 5, 2, 3, 4).reshape(B, C, D, h, w)
    assert x.max().item() <= float(bound) ** 2
    g = torch.Generator().manual_seed(12)
    wt = torch.randn(8, 32, 3, 3, 3, generator=g) * 0.05
    _check(x, wt, None, words, "fused cost volume")


# ---- conv_1_0: stride-2 split kernel (csrc/conv3d_s2_split.hip) ------------------------------------
def _split_host_s2(w):
    lib = _lib.load()
    w = w.to(torch.float32).contiguous()
    frag = torch.empty((27 * 2 * 64 * 8,), dtype=torch.int16)
    e = ctypes.c_int(0)
    st = lib.mvs_conv3d_s2_split_weights(_lib.ptr(w), _lib.ptr(frag), ctypes.byref(e))
    return st, frag.view(torch.float16).reshape(27, 2, 64, 8).to(torch.float64), e.value


def test_s2_split_weights_layout():
    g = torch.Generator().manual_seed(8)
    w = torch.randn(16, 32, 3, 3, 3, generator=g) * 0.03
    st, frag, ew = _split_host_s2(w)
    assert st == 0
    m = w.abs().max().item()
    assert m * 2.0 ** ew < 2 ** 14 <= 2 * m * 2.0 ** ew
    ws = w.double() * 2.0 ** ew
    for tap in (0, 5, 26):
        kz, ky, kx = tap // 9, (tap // 3) % 3, tap % 3
        hi = torch.zeros(16, 32, dtype=torch.float64)
        lo = torch.zeros(16, 32, dtype=torch.float64)
        for l in range(64):
            for j in range(8):
                hi[l & 15, 8 * (l >> 4) + j] = frag[tap, 0, l, j]
                lo[l & 15, 8 * (l >> 4) + j] = frag[tap, 1, l, j]
        ref = ws[:, :, kz, ky, kx]
        assert torch.equal(hi, ref.to(torch.float16).double())
        assert (hi + lo - ref).abs().max() <= 2.0 ** -22 * ref.abs().max() + 2.0 ** -24


@pytest.mark.gpu
@pytest.mark.parametrize("n", [(12, 16, 20), (15, 21, 37), (24, 33, 50)])
@pytest.mark.parametrize("bn", [False, True])
def test_s2_split_conv_on_live_region(n, bn):
    """conv_1_0 on forward_live's halo(B) (stride 2, padding n//2 + 1: windows leave the volume on
    every side), ragged output tiles, against float64 of the same volume and no worse than 1.5x the
    fp32 region kernel's / MIOpen's own error; the output region is channels-last."""
    from mvs_amd import model as M
    from mvs_amd.config import pad_outpad
    from mvs_amd.ops import CONV_S2, conv3d_region, conv_s2_split
    pad, _ = pad_outpad(*n)
    full = tuple((0, d - 1) for d in n)
    halo = M._grow(M._tconv_input_region(full, n, pad), n, 1)
    org = [lo for lo, _ in halo]
    size = [hi - lo + 1 for lo, hi in halo]
    g = torch.Generator().manual_seed(sum(n) + bn)
    B = 2
    x = torch.randn(B, 32, *n, generator=g).square()
    wt = torch.randn(16, 32, 3, 3, 3, generator=g) * 0.05
    p = (torch.rand(16, generator=g) + 0.5, torch.randn(16, generator=g), torch.randn(16, generator=g) * 0.1) if bn else None
    ref = torch.nn.functional.conv3d(x.double(), wt.double(), stride=2, padding=pad)
    if bn:
        sc, sh, mu = (t.double()[:, None, None, None] for t in p)
        ref = torch.clamp((ref - mu) * sc + sh, min=0.0)
    sl = tuple(slice(o, o + s) for o, s in zip(org, size))
    ref = ref[(slice(None), slice(None)) + sl].permute(0, 2, 3, 4, 1)          # channels-last region
    bdev = [t.to(DEV) for t in p] if bn else []
    with torch.no_grad():
        xc = _to_c4(x).to(DEV)
        y = conv_s2_split(xc, _bound_words(x).to(DEV), wt.to(DEV), list(n), org, size, list(pad), *bdev).cpu()
        w27 = wt.permute(2, 3, 4, 0, 1).reshape(27, 16, 32).contiguous().to(DEV)
        y32 = conv3d_region(xc, None, w27, CONV_S2, list(n), org, size, None, None, list(pad), *bdev, in_c4=True).cpu()
        yt = torch.nn.functional.conv3d(x.to(DEV), wt.to(DEV), stride=2, padding=pad)
        if bn:
            sc, sh, mu = (t.to(DEV)[:, None, None, None] for t in p)
            yt = torch.clamp((yt - mu) * sc + sh, min=0.0)
        yt = yt[(slice(None), slice(None)) + sl].permute(0, 2, 3, 4, 1).cpu()
    assert y.shape == ref.shape == y32.shape, (y.shape, ref.shape, y32.shape)
    scale = ref.abs().max().item()
    err = (y.double() - ref).abs().max().item()
    err32 = (y32.double() - ref).abs().max().item()
    errt = (yt.double() - ref).abs().max().item()
    print("s2 %s bn=%s: split %.3g, fp32 region kernel %.3g, MIOpen %.3g (scale %.3g)" % (n, bn, err, err32, errt, scale))
    assert err <= 1e-5 * scale, (err, scale)
    assert err <= 1.5 * max(err32, errt) + 1e-7 * scale, (err, err32, errt)


# ---- the split cost volume (mvs_cost_volume_fwd_c4_split, csrc/split.h) ---------------------------
def _fused_volumes(B=2, V=3, C=32, h=40, w=52, D=12, seed=11, scale=7.0):
    from cameras import camera_batch, depth_range, features
    from mvs_amd import ops
    K, R, T = camera_batch(B, V, h, w)
    d_min, d_int = depth_range(B, d_int=4.0, distinct=True)
    feat = (features(B * V, C, h, w, seed=seed) * scale).to(DEV)
    with torch.no_grad():
        c4, a4 = ops.cost_volume_c4_absmax(feat, K, R, T, d_min, d_int, B, V, 0, D, 25.0)
        sp, asp = ops.cost_volume_c4_split(feat, K, R, T, d_min, d_int, B, V, 0, D, 25.0)
    return c4, a4, sp, asp


@pytest.mark.gpu
def test_split_cost_volume_is_the_split_of_the_fp32_volume():
    """Every 16-byte element of the split volume is exactly (fp16(v 2^e), fp16(v 2^e - hi)) of the fp32
    channel-quad volume's values (same kernel arithmetic, split in the store), e from the bound words
    (the same words as the fp32 op's); unsplit gives the values back to 2^-22."""
    from mvs_amd import ops
    c4, a4, sp, asp = _fused_volumes()
    assert torch.equal(a4, asp)
    e = ops.split_exponent(asp)
    v = torch.ldexp(c4.double().cpu(), torch.tensor(float(e), dtype=torch.float64))
    hi = v.float().half()
    lo = (v - hi.double()).float().half()
    got = sp.cpu().view(torch.float16).reshape(sp.shape[:-1] + (2, 4))
    assert torch.equal(got[..., 0, :].view(torch.int16), hi.view(torch.int16))
    assert torch.equal(got[..., 1, :].view(torch.int16), lo.view(torch.int16))
    # to 2^-22 relative in fp16's normal range; below it lo is a subnormal (spacing 2^-24 scaled)
    back = ops.unsplit_cost_volume(sp, asp).cpu()
    assert ((back - c4.cpu()).abs() <= 2.0 ** -21 * c4.cpu().abs() + 2.0 ** (-24 - e)).all()


@pytest.mark.gpu
def test_split_consumers_read_the_split_volume_like_fp32():
    """conv_0_0 and conv_1_0 on the split volume: bit-identical to the same kernels converting the fp32
    volume themselves (the same operands reach the MFMAs); conv_2_0 on the region kernel reading the
    split volume: within 2^-21 relative of the input perturbation (fp32 re-formed as hi + lo)."""
    from mvs_amd import model as M
    from mvs_amd.config import pad_outpad
    from mvs_amd.ops import CONV_S2, conv3d_k3_split, conv3d_region, conv_s2_split
    c4, a4, sp, asp = _fused_volumes()
    n = tuple(c4.shape[2:5])
    g = torch.Generator().manual_seed(21)
    w0 = (torch.randn(8, 32, 3, 3, 3, generator=g) * 0.05).to(DEV)
    w1 = (torch.randn(16, 32, 3, 3, 3, generator=g) * 0.05).to(DEV)
    w2 = (torch.randn(32, 32, 3, 3, 3, generator=g) * 0.05).to(DEV)
    pad, _ = pad_outpad(*n)
    full = tuple((0, d - 1) for d in n)
    Bq = M._tconv_input_region(full, n, pad)
    h1 = M._grow(Bq, n, 1)
    h2 = M._grow(M._tconv_input_region(Bq, n, pad), n, 1)
    org = lambda r: [lo for lo, _ in r]
    size = lambda r: [hi - lo + 1 for lo, hi in r]
    with torch.no_grad():
        assert torch.equal(conv3d_k3_split(sp, asp, w0), conv3d_k3_split(c4, a4, w0))
        assert torch.equal(conv_s2_split(sp, asp, w1, list(n), org(h1), size(h1), list(pad)),
                           conv_s2_split(c4, a4, w1, list(n), org(h1), size(h1), list(pad)))
        w27 = w2.permute(2, 3, 4, 0, 1).reshape(27, 32, 32).contiguous()
        ys = conv3d_region(sp, None, w27, CONV_S2, list(n), org(h2), size(h2), None, None, list(pad), in_c4=True,
                           absmax=asp)
        yf = conv3d_region(c4, None, w27, CONV_S2, list(n), org(h2), size(h2), None, None, list(pad), in_c4=True)
    scale = yf.abs().max().item()
    assert (ys - yf).abs().max().item() <= 1e-6 * scale
