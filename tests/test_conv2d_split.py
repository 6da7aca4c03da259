"""The feature encoder's and refinement net's Conv2d layers on split-fp16 MFMA (csrc/conv2d_split.hip,
ops.conv2d_split; model.py:35-59 layers 2-8 and model.py:134-145's 32 -> 32 on the inference path) and
the bound words that scale their inputs (raised by conv2d_narrow.hip's epilogue for the first layer).

Parity: against torch's float64 convolution (CPU), with the error bounded by the fp32 direct kernel's
(ops.conv2d, one fp32 FMA per term) on the same inputs -- the split operands carry 22 significant bits,
the accumulation is fp32.  Bound words: every producer raises them to exactly max|y|.
"""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

DEV = torch.device("cuda", 0)
SHAPES = [(8, 8, 3, 1), (8, 16, 5, 2), (16, 16, 3, 1), (16, 32, 5, 2), (32, 32, 3, 1)]


def test_conv2d_split_fragments_host():
    """CPU: mvs_conv2d_split_weights lays out hi / lo parts as the header documents (32 / c_in taps per
    K-32 block, zero taps past k^2; c_out = 8 as [w_hi | w_lo] columns), the parts sum to w 2^ew within
    2^-21 relative, and max|w| 2^ew < 2^14."""
    from mvs_amd.ops import conv2d_split_fragments
    g = torch.Generator().manual_seed(11)
    for cin, cout, k, _ in SHAPES:
        w = torch.randn(cout, cin, k, k, generator=g) * 0.07
        frag, ew = conv2d_split_fragments(w, torch.device("cpu"))
        tpb, cpt = 32 // cin, cin // 8
        kb = -(-(k * k) // tpb)
        f = frag.view(torch.float16).double()
        rec = torch.zeros(cout, cin, kb * tpb, dtype=torch.float64)   # [co][ci][tap]
        if cout == 8:
            f = f.view(kb, 4, 16, 8)                                      # [kb][g][c][j]
            parts = f[:, :, :8] + f[:, :, 8:]                             # hi (columns < 8) + lo
            nbs = [(0, parts)]
        else:
            f = f.view(kb, cout // 16, 2, 4, 16, 8)                       # [kb][nb][part][g][c][j]
            nbs = [(nb, f[:, nb, 0] + f[:, nb, 1]) for nb in range(cout // 16)]
        for nb, parts in nbs:
            width = parts.shape[2]
            for b in range(kb):
                for gq in range(4):
                    tap, c0 = b * tpb + gq // cpt, 8 * (gq % cpt)
                    rec[nb * 16:nb * 16 + width, c0:c0 + 8, tap] = parts[b, gq]
        ref = w.double().reshape(cout, cin, k * k) * 2.0 ** ew
        assert w.abs().max().item() * 2.0 ** ew < 2.0 ** 14
        assert (rec[:, :, :k * k] - ref).abs().max().item() <= 2.0 ** -21 * ref.abs().max().item()
        if kb * tpb > k * k:   # the last block's taps past k^2 are zeros
            assert rec[:, :, k * k:].abs().max().item() == 0.0


def test_conv2d_split_rejects_bad_arguments():
    """CPU: argument checks run before any launch (no GPU needed): null input / weight / output / bound
    words, a misaligned fragment pointer, an unsupported shape."""
    import ctypes
    from mvs_amd import _lib
    lib = _lib.load()
    fake, odd, null = ctypes.c_void_p(4096), ctypes.c_void_p(4104), None
    args = lambda x, wf, y, xb, cin=8, cout=8, k=3, s=1: (x, wf, 0, y, 2, cin, cout, 64, 64, k, s, None, None,
                                                         None, xb, None, null)
    assert lib.mvs_conv2d_split_fwd(*args(null, fake, fake, fake)) == -1
    assert lib.mvs_conv2d_split_fwd(*args(fake, null, fake, fake)) == -1
    assert lib.mvs_conv2d_split_fwd(*args(fake, fake, null, fake)) == -1
    assert lib.mvs_conv2d_split_fwd(*args(fake, fake, fake, null)) == -1
    assert lib.mvs_conv2d_split_fwd(*args(fake, odd, fake, fake)) == -1
    w = (ctypes.c_float * (8 * 3 * 9))()
    frag = (ctypes.c_uint16 * 4096)()
    e = ctypes.c_int(0)
    assert lib.mvs_conv2d_split_weights(w, 3, 8, 3, frag, ctypes.byref(e)) == -1    # c_in 3: VALU kernel only
    assert lib.mvs_conv2d_split_weights(w, 8, 12, 3, frag, ctypes.byref(e)) == -1


def _bn(c, g):
    return (torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.1, torch.randn(c, generator=g) * 0.1)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("bn,amp,hw", [(True, 1.0, (37, 50)), (False, 1.0, (64, 80)), (True, 4e3, (40, 48)),
                                       (False, 3e-4, (33, 29))])
def test_conv2d_split_matches_torch(shape, bn, amp, hw):
    """conv2d_split on ragged and tile-aligned images (partial 16 x 16 / 16 x 8 tiles, odd widths: the
    scalar store path), inputs scaled by ``amp`` (the bound words carry the scale), with and without
    the eval BN + ReLU: max error <= 2x the fp32 direct kernel's + 1e-6 of the output scale, against
    float64 torch; the output bound words equal max|y| exactly."""
    from mvs_amd.ops import bound_words, conv2d, conv2d_split
    import torch.nn.functional as F
    cin, cout, k, s = shape
    g = torch.Generator().manual_seed(cin * 7 + cout + k + int(bn))
    x = torch.randn(2, cin, *hw, generator=g) * amp
    if bn:
        x = torch.relu(x)   # the encoder's inputs past the first layer are BN + ReLU outputs
    w = torch.randn(cout, cin, k, k, generator=g) * (1.0 / (cin * k * k) ** 0.5)
    p = _bn(cout, g) if bn else None
    ref = F.conv2d(x.double(), w.double(), stride=s, padding=k // 2)
    if bn:
        sc, sh, mu = (t.double().view(1, -1, 1, 1) for t in p)
        ref = torch.relu((ref - mu) * sc + sh)
    words = bound_words(2, DEV)
    xg = x.to(DEV)
    # the input's bound words from the fp32 kernel's epilogue (as the encoder's first layer raises
    # them): an identity-weight 3 x 3 conv (cin -> cin is a supported shape) copies x exactly
    eye = torch.zeros(cin, cin, 3, 3)
    for c in range(cin):
        eye[c, c, 1, 1] = 1.0
    xc = conv2d(xg, eye.to(DEV), 1, y_bound=words[0])
    assert torch.equal(xc.cpu(), x)
    assert words[0].max().view(torch.float32).item() == x.abs().max().item()
    pg = [t.to(DEV) for t in p] if bn else []
    y = conv2d_split(xc, w.to(DEV), s, words[0], words[1], *pg).cpu().double()
    y32 = conv2d(xg, w.to(DEV), s, *pg).cpu().double()
    scale = ref.abs().max().item()
    err, err32 = (y - ref).abs().max().item(), (y32 - ref).abs().max().item()
    assert err <= 2 * err32 + 1e-6 * scale, (err, err32, scale)
    assert words[1].max().view(torch.float32).item() == y.abs().max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["encoder", "refine"])
def test_stack_split_path_matches_fp32_path(which, monkeypatch):
    """FeatureEncoder / DepthRefinement in eval mode: the split-fp16 stack (split_f16 on: the opt-in
    arithmetic) against the fp32 direct-kernel stack (the default) and float64 modules: the split path's
    error is at most 2x the fp32 path's + 1e-6 of the output scale."""
    from mvs_amd.model import DepthRefinement, FeatureEncoder
    torch.manual_seed(0)
    net, shape = (FeatureEncoder(), (3, 3, 96, 136)) if which == "encoder" else (DepthRefinement(), (2, 4, 40, 56))
    for mod in net.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_mean.uniform_(-0.5, 0.5)
            mod.running_var.uniform_(0.5, 2.0)
            mod.weight.data.uniform_(0.5, 1.5)
            mod.bias.data.uniform_(-0.5, 0.5)
    net = net.eval()
    x = torch.randn(shape, generator=torch.Generator().manual_seed(5))
    with torch.no_grad():
        ref = net.double()(x.double())
        net = net.float().to(DEV)
        net.split_f16 = True
        y = net(x.to(DEV)).cpu().double()
        net.split_f16 = False
        y32 = net(x.to(DEV)).cpu().double()
        monkeypatch.setenv("MVS_CONV2D_F16", "0")   # the kill switch of the split stack
        net.split_f16 = True
        assert torch.equal(net(x.to(DEV)).cpu().double(), y32)
    scale = ref.abs().max().item()
    err, err32 = (y - ref).abs().max().item(), (y32 - ref).abs().max().item()
    assert err <= 2 * err32 + 1e-6 * scale, (err, err32, scale)
