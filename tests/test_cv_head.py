"""The cost volume consumed where it is formed (csrc/cv_head.hip, ops.cost_volume_head).

Two modes of one kernel, both in the opt-in split-fp16 arithmetic (MVSConfig(arithmetic="split_f16")).
The split head (ops.split_head, PRESPLIT) reads the materialised split volume and runs conv_0_0 and
conv_1_0 in one pass over it.  The fused head (MVS_CV_HEAD=1, ops.cost_volume_head) forms the variance on
chip as well, so the volume is never written.  Its gathering producers corrupted the .z / .w halves of
a few items' variance in a schedule-dependent share of launches (rounds 4-6; up to every launch in some
builds): the instructions involved are the packed fp32 VALU ops of the gather / variance code, and the
head now ships without them (csrc/cv_head.hip built with the packed-fp32-ops feature off,
tests/test_head_isa.py rule 3) -- 0 of 900 launches differ at the bench geometry and a small one, and a
build that failed every launch fails none without packed fp32.  Its bit-equality tests
below are strict again, with a 20-launch repeatability test at the bench geometry.

The fused head forms the variance of homography_warping + assemble_cost_volume (homography.py:6-92,
costvolume.py:3-16) on chip and applies conv_0_0 + BN_0 + ReLU (model.py:101) and conv_1_0 + BN_1 +
ReLU (model.py:103) to it.  It uses the materialising path's arithmetic operand for operand and MFMA
for MFMA, so its outputs must be BIT-EQUAL to that path: the split cost volume
(mvs_cost_volume_fwd_c4_split) fed to the split-fp16 conv_0_0 (mvs_conv3d_k3_split_fwd) and conv_1_0
(mvs_conv3d_s2_split_fwd), whose own parity against float64 and the oracle is pinned in
test_split_conv.py / test_gpu_configs.py.  The split volume the head stores on conv_2_0's input box
must equal the materialised one there.
"""
import os

import numpy as np
import pytest
import torch

DEV = torch.device("cuda", 0)


def _regions(n, pad):
    from mvs_amd import model as M
    full = tuple((0, d - 1) for d in n)
    B = M._tconv_input_region(full, n, pad)
    C2 = M._tconv_input_region(B, n, pad)
    h1, h2 = M._grow(B, n, 1), M._grow(C2, n, 1)
    lo = [max(2 * a - p, 0) for (a, _), p in zip(h2, pad)]
    hi = [min(2 * b - p + 2, d - 1) + 1 for (_, b), p, d in zip(h2, pad, n)]
    return h1, lo, hi


def test_bare_split_volume_is_rejected():
    """CPU: a split (int32) channel-quad volume without its bound words raises a clear error instead
    of silently dropping to another scale (the bound travels in ops.BoundCostVolume)."""
    from mvs_amd.model import CostVolumeReg
    from mvs_amd.config import pad_outpad
    reg = CostVolumeReg(pad=pad_outpad(8, 8, 8)[0], outpad=pad_outpad(8, 8, 8)[1]).eval()
    with pytest.raises(ValueError, match="bound words"):
        reg(torch.zeros((1, 8, 8, 8, 8, 4), dtype=torch.int32))


def test_bound_cost_volume_travels_with_its_bound():
    """CPU: BoundCostVolume keeps data and bound together through clone(); to_ncdhw() is the reference
    layout of the channel-quad values."""
    from mvs_amd.ops import BoundCostVolume
    q = torch.randn(2, 3, 4, 5, 6, 4)
    b = BoundCostVolume(q, torch.zeros(8, dtype=torch.int32))
    c = b.clone()
    assert c.data is not q and torch.equal(c.data, q) and torch.equal(c.absmax, b.absmax)
    ref = q.permute(0, 1, 5, 2, 3, 4).reshape(2, 12, 4, 5, 6)
    assert torch.equal(b.to_ncdhw(), ref)
    with pytest.raises(ValueError):
        BoundCostVolume(q, torch.zeros(4, dtype=torch.int32))


def test_partial_cost_volume_refuses_whole_volume_views():
    """CPU: a boxed (partial) volume -- what the fused head stores -- keeps its box through clone()
    and raises instead of returning values it does not hold (no silent uninitialised data)."""
    from mvs_amd.ops import BoundCostVolume
    q = torch.zeros(1, 8, 3, 4, 5, 4, dtype=torch.int32)
    b = BoundCostVolume(q, torch.zeros(8, dtype=torch.int32), [1, 2, 3], [8, 8, 8])
    assert b.partial and b.box_region() == ([1, 2, 3], [3, 4, 5])
    assert b.clone().box_region() == b.box_region()
    for f in (b.quads, b.to_ncdhw):
        with pytest.raises(ValueError, match="partial"):
            f()
    with pytest.raises(ValueError, match="outside"):
        BoundCostVolume(q, torch.zeros(8, dtype=torch.int32), [6, 0, 0], [8, 8, 8])
    with pytest.raises(ValueError):
        BoundCostVolume(q, torch.zeros(8, dtype=torch.int32), [0, 0, 0], None)


@pytest.mark.gpu
@pytest.mark.parametrize("B,V,D,h,w", [(2, 3, 16, 32, 48), (1, 2, 20, 24, 40), (1, 3, 100, 36, 44),
                                       (2, 3, 48, 28, 64), (1, 2, 20, 25, 32), (1, 3, 16, 29, 41)])
def test_head_is_bit_equal_to_the_split_path(B, V, D, h, w):
    """y0, y1 and the stored box are bit-equal to cost_volume_c4_split -> conv3d_k3_split /
    conv_s2_split; geometries with one and several 48-plane chunks (a partial last one at D = 100),
    V = 2 and 3, widths / heights not multiples of the 16 x 4 tile; both, one (25 x 32: x only, 24 x 40:
    y only) and neither (29 x 41) of w % 16 == 0, h % 4 == 0 (the edge tile column / row that owns only
    the last stride-2 window)."""
    from cameras import camera_batch, depth_range
    from mvs_amd import ops
    from mvs_amd.config import pad_outpad
    C = 32
    pad = list(pad_outpad(D, h, w)[0])
    assert all(p % 2 for p in pad)
    n = (D, h, w)
    h1, lo, hi = _regions(n, pad)
    K, R, T = camera_batch(B, V, h, w)
    d_min, d_int = depth_range(B, d_int=200.0 / D)
    g = torch.Generator().manual_seed(D + h + w)
    feat = torch.randn(B * V, C, h, w, generator=g).to(DEV)
    w0 = (torch.randn(8, 32, 3, 3, 3, generator=g) * 0.1).to(DEV)
    w1 = (torch.randn(16, 32, 3, 3, 3, generator=g) * 0.1).to(DEV)
    bn0 = [(torch.rand(8, generator=g) + 0.5).to(DEV), (torch.randn(8, generator=g) * 0.1).to(DEV),
           (torch.randn(8, generator=g) * 0.1).to(DEV)]
    bn1 = [(torch.rand(16, generator=g) + 0.5).to(DEV), (torch.randn(16, generator=g) * 0.1).to(DEV),
           (torch.randn(16, generator=g) * 0.1).to(DEV)]
    org, size = [a for a, _ in h1], [b - a + 1 for a, b in h1]
    with torch.no_grad():
        scv, absmax = ops.cost_volume_c4_split(feat, K, R, T, d_min, d_int, B, V, 0, D, 25.0)
        y0_ref = ops.conv3d_k3_split(scv, absmax, w0, *bn0)
        y1_ref = ops.conv_s2_split(scv, absmax, w1, list(n), org, size, pad, *bn1)
        y0, y1, box, am = ops.cost_volume_head(feat, K, R, T, d_min, d_int, B, V, 0, D, 25.0, w0, *bn0, w1, *bn1,
                                               pad, org, size, lo, hi)
        torch.cuda.synchronize()
    assert torch.equal(am, absmax)
    assert torch.equal(y0, y0_ref), (y0 - y0_ref).abs().max().item()
    assert torch.equal(y1, y1_ref), (y1 - y1_ref).abs().max().item()
    sl = (slice(None), slice(None)) + tuple(slice(a, b) for a, b in zip(lo, hi))
    assert list(box.shape) == [B, 8] + [b - a for a, b in zip(lo, hi)] + [4]   # only the box is allocated
    assert torch.equal(box, scv[sl])
    # without BN epilogues (raw convolution values) as well
    with torch.no_grad():
        y0n, y1n, _, _ = ops.cost_volume_head(feat, K, R, T, d_min, d_int, B, V, 0, D, 25.0, w0, None, None, None,
                                              w1, None, None, None, pad, org, size, lo, hi)
        assert torch.equal(y0n, ops.conv3d_k3_split(scv, absmax, w0))
        assert torch.equal(y1n, ops.conv_s2_split(scv, absmax, w1, list(n), org, size, pad))


@pytest.mark.gpu
def test_mvsnet_head_equals_split_volume_path():
    """MVSNet.forward with the opt-in fused head (MVS_CV_HEAD=1) gives the same depth maps, bit for
    bit, as the same network fed the materialised split volume (the default), at cfg 1's geometry
    with B = 2."""
    from cameras import camera_batch, depth_range
    from mvs_amd.config import MVSConfig
    from mvs_amd.model import MVSNet
    B, V, D, H, W = 2, 3, 48, 512, 640
    torch.manual_seed(0)
    net = MVSNet(MVSConfig(d_num=D, in_h=H, in_w=W, arithmetic="split_f16")).to(DEV).eval()
    K, R, T = camera_batch(B, V, H // 4, W // 4)
    d_min, d_int = depth_range(B)
    img = torch.randn(B * V, 3, H, W, generator=torch.Generator().manual_seed(5)).to(DEV)
    import mvs_amd.costvolume as cvmod
    calls = []
    orig = cvmod.DeferredCostVolume.head

    def spy(self, *a, **kw):
        calls.append(1)
        return orig(self, *a, **kw)
    with torch.no_grad():
        cvmod.DeferredCostVolume.head = spy
        os.environ["MVS_CV_HEAD"] = "1"
        try:
            d_head, r_head = net(img, K, R, T, d_min, d_int, B, V)
        finally:
            cvmod.DeferredCostVolume.head = orig
            os.environ.pop("MVS_CV_HEAD")
        d_split, r_split = net(img, K, R, T, d_min, d_int, B, V)
    assert calls == [1]
    assert torch.equal(d_head, d_split) and torch.equal(r_head, r_split)


@pytest.mark.gpu
def test_mvsnet_split_head_equals_separate_convolutions():
    """MVSNet.forward's default eval path (split volume -> ops.split_head) gives the same depth maps,
    bit for bit, as conv3d_k3_split + conv_s2_split (MVS_SPLIT_HEAD=0), and calls the split head once
    per forward, at cfg 1's geometry with B = 2 and V = 5 (any view count: the head reads the volume)."""
    from cameras import camera_batch, depth_range
    from mvs_amd import ops
    from mvs_amd.config import MVSConfig
    from mvs_amd.model import MVSNet
    B, V, D, H, W = 2, 5, 48, 512, 640
    torch.manual_seed(0)
    net = MVSNet(MVSConfig(d_num=D, in_h=H, in_w=W, arithmetic="split_f16")).to(DEV).eval()
    K, R, T = camera_batch(B, V, H // 4, W // 4)
    d_min, d_int = depth_range(B)
    img = torch.randn(B * V, 3, H, W, generator=torch.Generator().manual_seed(6)).to(DEV)
    kinds = []
    with torch.no_grad():
        ops.KERNEL_EVENT_HOOK = lambda kind: (kinds.append(kind), (torch.cuda.Event(), torch.cuda.Event()))[1]
        try:
            d_sh, r_sh = net(img, K, R, T, d_min, d_int, B, V)
        finally:
            ops.KERNEL_EVENT_HOOK = None
        os.environ["MVS_SPLIT_HEAD"] = "0"
        try:
            d_sep, r_sep = net(img, K, R, T, d_min, d_int, B, V)
        finally:
            os.environ.pop("MVS_SPLIT_HEAD")
    assert kinds.count("split_head") == 1 and "cv_head" not in kinds
    assert torch.equal(d_sh, d_sep) and torch.equal(r_sh, r_sep)


@pytest.mark.gpu
@pytest.mark.parametrize("B,D,h,w", [(2, 16, 32, 48), (1, 20, 24, 40), (1, 100, 36, 44), (1, 20, 25, 32),
                                     (1, 16, 29, 41), (4, 192, 128, 160)])
def test_split_head_is_bit_equal_and_repeatable(B, D, h, w):
    """ops.split_head (mvs_split_head_fwd: the head's consumer half fed from a materialised split
    volume) returns y0 / y1 bit-equal to conv3d_k3_split / conv_s2_split, with and without BN
    epilogues, and the same bits on every one of 10 launches."""
    from cameras import camera_batch, depth_range
    from mvs_amd import ops
    from mvs_amd.config import pad_outpad
    n = (D, h, w)
    if D == 16:   # a plain padding-1 convolution over its whole output as well
        pad = [1, 1, 1]
        org, size = [0, 0, 0], [(d + 2 * p - 3) // 2 + 1 for d, p in zip(n, pad)]
    else:         # the model's conv_1_0 (config.py:20 padding) on the region deconv_1_0 reads
        pad = list(pad_outpad(D, h, w)[0])
        h1 = _regions(n, pad)[0]
        org, size = [a for a, _ in h1], [b - a + 1 for a, b in h1]
    K, R, T = camera_batch(B, 2, h, w)
    d_min, d_int = depth_range(B, d_int=200.0 / D)
    g = torch.Generator().manual_seed(D + h + w + 1)
    feat = torch.randn(B * 2, 32, h, w, generator=g).to(DEV)
    w0 = (torch.randn(8, 32, 3, 3, 3, generator=g) * 0.1).to(DEV)
    w1 = (torch.randn(16, 32, 3, 3, 3, generator=g) * 0.1).to(DEV)
    bn0 = [(torch.rand(8, generator=g) + 0.5).to(DEV), (torch.randn(8, generator=g) * 0.1).to(DEV),
           (torch.randn(8, generator=g) * 0.1).to(DEV)]
    bn1 = [(torch.rand(16, generator=g) + 0.5).to(DEV), (torch.randn(16, generator=g) * 0.1).to(DEV),
           (torch.randn(16, generator=g) * 0.1).to(DEV)]
    with torch.no_grad():
        scv, absmax = ops.cost_volume_c4_split(feat, K, R, T, d_min, d_int, B, 2, 0, D, 25.0)
        for bn in (True, False):
            b0, b1 = (bn0, bn1) if bn else ([None] * 3, [None] * 3)
            y0_ref = ops.conv3d_k3_split(scv, absmax, w0, *b0)
            y1_ref = ops.conv_s2_split(scv, absmax, w1, list(n), org, size, pad, *b1)
            bad = 0
            for _ in range(10 if bn else 2):
                y0, y1 = ops.split_head(scv, absmax, w0, *b0, w1, *b1, pad, org, size)
                torch.cuda.synchronize()
                bad += not (torch.equal(y0, y0_ref) and torch.equal(y1, y1_ref))
            assert bad == 0, ("bn" if bn else "raw", bad, (y0 - y0_ref).abs().max().item(),
                              (y1 - y1_ref).abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("V", [2, 3])
def test_fused_head_repeatable_at_the_bench_geometry(V):
    """20 launches of the fused head at cfg 2's geometry (B = 4, 192 x 128 x 160, BN epilogues), every one
    bit-equal to the materialising split path on y0, y1 and the box (round 5: 15-20 of 20 launches
    differed here)."""
    from cameras import camera_batch, depth_range
    from mvs_amd import ops
    from mvs_amd.config import pad_outpad
    B, D, h, w = 4, 192, 128, 160
    pad = list(pad_outpad(D, h, w)[0])
    n = (D, h, w)
    h1, lo, hi = _regions(n, pad)
    K, R, T = camera_batch(B, V, h, w)
    d_min, d_int = depth_range(B, d_int=200.0 / D)
    g = torch.Generator().manual_seed(7 + V)
    feat = torch.randn(B * V, 32, h, w, generator=g).to(DEV)
    w0 = (torch.randn(8, 32, 3, 3, 3, generator=g) * 0.1).to(DEV)
    w1 = (torch.randn(16, 32, 3, 3, 3, generator=g) * 0.1).to(DEV)
    bn0 = [(torch.rand(8, generator=g) + 0.5).to(DEV), (torch.randn(8, generator=g) * 0.1).to(DEV),
           (torch.randn(8, generator=g) * 0.1).to(DEV)]
    bn1 = [(torch.rand(16, generator=g) + 0.5).to(DEV), (torch.randn(16, generator=g) * 0.1).to(DEV),
           (torch.randn(16, generator=g) * 0.1).to(DEV)]
    org, size = [a for a, _ in h1], [b - a + 1 for a, b in h1]
    sl = (slice(None), slice(None)) + tuple(slice(a, b) for a, b in zip(lo, hi))
    with torch.no_grad():
        scv, absmax = ops.cost_volume_c4_split(feat, K, R, T, d_min, d_int, B, V, 0, D, 25.0)
        ref = (ops.conv3d_k3_split(scv, absmax, w0, *bn0), ops.conv_s2_split(scv, absmax, w1, list(n), org, size, pad, *bn1),
               scv[sl].clone())
        del scv
        bad = []
        for it in range(20):
            y0, y1, box, _ = ops.cost_volume_head(feat, K, R, T, d_min, d_int, B, V, 0, D, 25.0, w0, *bn0, w1, *bn1,
                                                  pad, org, size, lo, hi)
            torch.cuda.synchronize()
            diff = [not torch.equal(a, b) for a, b in zip((y0, y1, box), ref)]
            if any(diff):
                bad.append((it, diff))
    assert not bad, "launches differing from the split path (y0, y1, box): %s" % bad


@pytest.mark.gpu
@pytest.mark.parametrize("bn_shift", [0.1, 50.0])
def test_split_head_bound_words_cover_every_output(bn_shift):
    """ops.split_head raises y1's bound words (the split-fp16 conv_1_1's input scale) to max |y1| over the
    WHOLE region, including the all-padding windows the faces launch fills with relu(BN_1(0)) (ADVICE r5:
    with a large positive BN shift those constants are the region's maximum)."""
    from cameras import camera_batch, depth_range
    from mvs_amd import ops
    from mvs_amd.config import pad_outpad
    from mvs_amd.ops import bound_words
    B, D, h, w = 1, 48, 128, 160
    pad = list(pad_outpad(D, h, w)[0])
    n = (D, h, w)
    h1 = _regions(n, pad)[0]
    org, size = [a for a, _ in h1], [b - a + 1 for a, b in h1]
    K, R, T = camera_batch(B, 2, h, w)
    d_min, d_int = depth_range(B, d_int=200.0 / D)
    g = torch.Generator().manual_seed(11)
    feat = torch.randn(B * 2, 32, h, w, generator=g).to(DEV)
    w0 = (torch.randn(8, 32, 3, 3, 3, generator=g) * 0.1).to(DEV)
    # conv_1_0 weights <= 0 on a variance (>= 0): every interior window's value is <= 0, so with a positive
    # BN shift relu(BN_1(0)) of the all-padding windows is the region's maximum
    w1 = -(torch.randn(16, 32, 3, 3, 3, generator=g) * 0.1).abs().to(DEV)
    bn0 = [torch.ones(8, device=DEV), torch.zeros(8, device=DEV), torch.zeros(8, device=DEV)]
    bn1 = [torch.ones(16, device=DEV), torch.full((16,), bn_shift, device=DEV), torch.zeros(16, device=DEV)]
    with torch.no_grad():
        scv, absmax = ops.cost_volume_c4_split(feat, K, R, T, d_min, d_int, B, 2, 0, D, 25.0)
        words = bound_words(1, DEV)[0]
        y0, y1 = ops.split_head(scv, absmax, w0, *bn0, w1, *bn1, pad, org, size, words)
        torch.cuda.synchronize()
    got = float(words.cpu().numpy().view(np.float32).max())
    assert got == y1.abs().max().item(), (got, y1.abs().max().item())
