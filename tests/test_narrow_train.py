"""GPU: the narrow full-volume convolutions under autograd (mvs_amd/narrow_train.py: conv_0_0
Conv3d(32, 8) and conv_out Conv3d(8, 1), model.py:101,124, in train.py:103's loss.backward) against
float64 torch autograd: output, input gradient and weight gradient within fp32 accumulation error
(|err| <= 1e-5 x the same sum over absolute values), the weight gradient bit-reproducible."""
import pytest
import torch
import torch.nn.functional as F

DEV = torch.device("cuda", 0) if torch.cuda.is_available() else None


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,shape", [(32, 8, (2, 8, 12, 40)), (8, 1, (1, 7, 37, 53)), (32, 8, (1, 5, 9, 33)),
                                            (16, 8, (2, 4, 8, 32)), (8, 8, (1, 9, 17, 70)), (8, 1, (3, 1, 1, 1))])
def test_narrow_conv_autograd_matches_float64(cin, cout, shape):
    from mvs_amd import narrow_train
    b, d, h, w = shape
    g = torch.Generator().manual_seed(cin * 100 + sum(shape))
    x = torch.randn(b, cin, d, h, w, generator=g)
    wt = torch.randn(cout, cin, 3, 3, 3, generator=g) * 0.1
    gy = torch.randn(b, cout, d, h, w, generator=g)
    conv = torch.nn.Conv3d(cin, cout, 3, padding=1, bias=False).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(wt)
    xg = x.to(DEV).requires_grad_(True)
    assert narrow_train.applies(conv, xg)
    y = narrow_train.conv3d(conv, xg)
    (y * gy.to(DEV)).sum().backward()
    x64, w64 = x.double().requires_grad_(True), wt.double().requires_grad_(True)
    y64 = F.conv3d(x64, w64, padding=1)
    (y64 * gy.double()).sum().backward()
    xa, wa = x.double().abs().requires_grad_(True), wt.double().abs().requires_grad_(True)
    ya = F.conv3d(xa, wa, padding=1)
    (ya * gy.double().abs()).sum().backward()
    for name, got, ref, bound in (("y", y.detach(), y64.detach(), ya.detach()), ("gx", xg.grad, x64.grad, xa.grad),
                                  ("gw", conv.weight.grad, w64.grad, wa.grad)):
        err = (got.double().cpu() - ref).abs()
        assert bool((err <= 1e-5 * bound + 1e-30).all()), "%s: max err %.3g" % (name, err.max().item())
    from mvs_amd.ops import conv3d_k3_wgrad
    a = conv3d_k3_wgrad(xg.detach(), gy.to(DEV))
    assert torch.equal(a, conv3d_k3_wgrad(xg.detach(), gy.to(DEV)))
    assert torch.equal(a, conv.weight.grad)


@pytest.mark.gpu
def test_narrow_conv_autograd_at_cfg2_conv0_shape():
    """conv_0_0's weight gradient at the cfg-2 volume (B=4, 32 x 192 x 128 x 160): against a float64
    reference of 6 of its 6,912 entries (per-tap dot products of the whole volume), within 1e-5 of the
    absolute sums."""
    from mvs_amd.ops import conv3d_k3_wgrad
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn(4, 32, 192, 128, 160, device=DEV, generator=g)
    gy = torch.randn(4, 8, 192, 128, 160, device=DEV, generator=g)
    dw = conv3d_k3_wgrad(x, gy)
    xp = F.pad(x, (1, 1, 1, 1, 1, 1))
    for co, ci, t in ((0, 0, 0), (7, 31, 26), (3, 17, 13), (5, 2, 4), (1, 30, 22), (6, 9, 8)):
        kz, ky, kx = t // 9, (t // 3) % 3, t % 3
        xs = xp[:, ci, kz:kz + 192, ky:ky + 128, kx:kx + 160]
        ref = (gy[:, co].double() * xs.double()).sum().item()
        bound = (gy[:, co].double().abs() * xs.double().abs()).sum().item()
        assert abs(dw[co, ci, kz, ky, kx].item() - ref) <= 1e-5 * bound, (co, ci, t)


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,k,s,hw", [(3, 8, 3, 1, (37, 53)), (8, 16, 5, 2, (40, 50)), (16, 32, 5, 2, (20, 26)),
                                             (32, 32, 3, 1, (19, 23))])
def test_encoder_conv2d_hip_forward_taps_backward(cin, cout, k, s, hw):
    """The encoder's Conv2d under autograd (tap_gemm.conv2d_hip_fwd: the HIP forward kernel, per-tap-GEMM
    backward) against float64 autograd: output and both gradients within 1e-5 of the absolute sums."""
    from mvs_amd import tap_gemm
    from mvs_amd.ops import conv2d_supported
    g = torch.Generator().manual_seed(cin * 7 + k)
    conv = torch.nn.Conv2d(cin, cout, k, stride=s, padding=k // 2, bias=False).to(DEV)
    if not conv2d_supported(conv):
        pytest.skip("not a reference layer shape")
    x = torch.randn((2, cin) + hw, generator=g)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(cout, cin, k, k, generator=g) * 0.1)
    xg = x.to(DEV).requires_grad_(True)
    y = tap_gemm.conv2d_hip_fwd(xg, conv)
    gy = torch.randn(y.shape, generator=g)
    (y * gy.to(DEV)).sum().backward()
    w = conv.weight.detach().cpu().double()
    x64, w64 = x.double().requires_grad_(True), w.clone().requires_grad_(True)
    (F.conv2d(x64, w64, stride=s, padding=k // 2) * gy.double()).sum().backward()
    xa, wa = x.double().abs().requires_grad_(True), w.abs().requires_grad_(True)
    ya = F.conv2d(xa, wa, stride=s, padding=k // 2)
    (ya * gy.double().abs()).sum().backward()
    y64 = F.conv2d(x.double(), w, stride=s, padding=k // 2)
    for name, got, ref, bound in (("y", y.detach(), y64, ya.detach()), ("gx", xg.grad, x64.grad, xa.grad),
                                  ("gw", conv.weight.grad, w64.grad, wa.grad)):
        err = (got.double().cpu() - ref).abs()
        assert bool((err <= 1e-5 * bound + 1e-30).all()), "%s: max err %.3g" % (name, err.max().item())


@pytest.mark.gpu
def test_region_convs_hip_forward_match_tap_gemms():
    """mvs_amd/region_train.py (training's region convolutions: HIP region-kernel forward, per-tap-GEMM
    backward) against tap_gemm's box convolutions on the same inputs at the live geometry of a
    (24, 20, 26) volume: outputs within fp32 accumulation error, input and weight gradients bit-equal
    (the same backward on the same saved operands)."""
    from mvs_amd import region_train, tap_gemm
    from mvs_amd.config import pad_outpad
    from mvs_amd.model import _crop_pad, _grow, _tconv_input_region
    n = (24, 20, 26)
    pad, _ = pad_outpad(*n)
    full = tuple((0, d - 1) for d in n)
    M = _tconv_input_region(full, n, pad)
    R1, R2 = _grow(M, n, 1), _grow(M, n, 2)
    g = torch.Generator().manual_seed(5)

    def check(fn_hip, fn_taps, inputs):
        outs, grads = [], []
        gy = None
        for fn in (fn_hip, fn_taps):
            xs = [t.detach().clone().to(DEV).requires_grad_(True) for t in inputs]
            y = fn(*xs)
            if gy is None:
                gy = torch.randn(y.shape, generator=g).to(DEV)
            (y * gy).sum().backward()
            outs.append(y.detach())
            grads.append([t.grad for t in xs])
        scale = outs[1].abs().max().item() + 1e-30
        assert (outs[0] - outs[1]).abs().max().item() <= 1e-5 * scale
        for a, b in zip(*grads):
            assert torch.equal(a, b)

    # stride-2 stacked conv_k_0 over R2 from the whole volume
    x = torch.randn(2, 32, *n, generator=g)
    w = torch.randn(112, 32, 3, 3, 3, generator=g) * 0.05
    pl, size = [], []
    for (lo, hi), p in zip(R2, pad):
        pl.append(max(2 * lo - p, 0) - (2 * lo - p))
        size.append(hi - lo + 1)
    check(lambda a, b: region_train.s2_box(a, b, R2, pad, tuple(pl), region_train.S2_SPLITS),
          lambda a, b: tap_gemm.conv3d_box(a, b, 2, tuple(pl), tuple(size)), [x, w])
    # stride-1 on a padded crop
    for c in (16, 32, 64):
        xin = torch.randn(2, c, *[hi - lo + 3 for lo, hi in R1], generator=g)
        w1 = torch.randn(c, c, 3, 3, 3, generator=g) * 0.05
        check(region_train.s1_valid, lambda a, b: tap_gemm.conv3d(a, b, 1, 0), [xin, w1])
    # transposed, M -> the full box
    for ci, co in region_train.T2_SHAPES:
        xm = torch.randn(2, ci, *[hi - lo + 1 for lo, hi in M], generator=g)
        wt = torch.randn(ci, co, 3, 3, 3, generator=g) * 0.05
        crop = tuple(lo - (2 * xlo - p) for (xlo, _), (lo, _), p in zip(M, full, pad))
        check(lambda a, b: region_train.t2_box(a, b, M, full, pad, n, crop),
              lambda a, b: tap_gemm.conv_transpose3d_box(a, b, 2, crop, n), [xm, wt])
