"""mvs_amd/tap_gemm.py (the training path's Conv3d / ConvTranspose3d as per-tap GEMMs with their own
backward) against PyTorch's autograd of F.conv3d / F.conv_transpose3d in float64 on the CPU: outputs,
input gradients and weight gradients, for the regulariser's shapes (stride 1 padding 1; stride 2
padding n//2 + 1; transposed stride 2 with output padding), odd and even extents, extents of 1-3
(parity grids with an empty parity) and paddings 0 / 1."""
import pytest
import torch
import torch.nn.functional as F

from mvs_amd import tap_gemm


def _grads(fn, x, w, gy):
    x = x.clone().requires_grad_(True)
    w = w.clone().requires_grad_(True)
    y = fn(x, w)
    (y * gy).sum().backward()
    return y.detach(), x.grad, w.grad


@pytest.mark.parametrize("n", [(5, 6, 7), (8, 9, 10), (2, 3, 1)])
@pytest.mark.parametrize("stride,pad", [(1, 1), (2, None), (2, 1), (1, 0)])
def test_conv3d_taps_autograd(n, stride, pad):
    g = torch.Generator().manual_seed(sum(n) + stride)
    p = tuple(d // 2 + 1 for d in n) if pad is None else pad
    if any(d + 2 * pp < 3 for d, pp in zip(n, p if isinstance(p, tuple) else (p,) * 3)):
        pytest.skip("kernel larger than the padded input")
    x = torch.randn(2, 5, *n, generator=g, dtype=torch.float64)
    w = torch.randn(3, 5, 3, 3, 3, generator=g, dtype=torch.float64)
    y_ref = F.conv3d(x, w, stride=stride, padding=p)
    gy = torch.randn(y_ref.shape, generator=g, dtype=torch.float64)
    ref = _grads(lambda a, b: F.conv3d(a, b, stride=stride, padding=p), x, w, gy)
    got = _grads(lambda a, b: tap_gemm.conv3d(a, b, stride, p), x, w, gy)
    for a, b in zip(got, ref):
        torch.testing.assert_close(a, b, rtol=1e-11, atol=1e-11)


@pytest.mark.parametrize("n", [(5, 6, 7), (8, 9, 10), (2, 3, 1)])
def test_conv_transpose3d_taps_autograd(n):
    g = torch.Generator().manual_seed(sum(n))
    p = tuple(d // 2 + 1 for d in n)
    op = tuple((d + 1) % 2 for d in n)
    x = torch.randn(2, 4, *n, generator=g, dtype=torch.float64)
    w = torch.randn(4, 3, 3, 3, 3, generator=g, dtype=torch.float64)
    f_ref = lambda a, b: F.conv_transpose3d(a, b, stride=2, padding=p, output_padding=op)
    y_ref = f_ref(x, w)
    gy = torch.randn(y_ref.shape, generator=g, dtype=torch.float64)
    ref = _grads(f_ref, x, w, gy)
    got = _grads(lambda a, b: tap_gemm.conv_transpose3d(a, b, 2, p, op), x, w, gy)
    for a, b in zip(got, ref):
        torch.testing.assert_close(a, b, rtol=1e-11, atol=1e-11)


def test_conv_module_dispatch():
    c = torch.nn.Conv3d(3, 2, 3, stride=2, padding=2, bias=False).double()
    t = torch.nn.ConvTranspose3d(2, 3, 3, stride=2, padding=2, output_padding=1, bias=False).double()
    x = torch.randn(1, 3, 6, 7, 8, dtype=torch.float64)
    torch.testing.assert_close(tap_gemm.conv_module(c, x), c(x), rtol=1e-12, atol=1e-12)
    z = torch.randn(1, 2, 4, 5, 6, dtype=torch.float64)
    torch.testing.assert_close(tap_gemm.conv_module(t, z), t(z), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("n,pad_lo,out", [((9, 7, 11), (2, 0, 3), (5, 4, 6)), ((6, 5, 8), (1, 1, 1), (4, 3, 5)),
                                          ((7, 7, 7), (0, 2, 1), (2, 6, 4))])
def test_conv3d_box_matches_sliced_padded_conv(n, pad_lo, out):
    """tap_gemm.conv3d_box: a box of a padded stride-2 convolution's output as a dense tensor, values
    and gradients against F.conv3d on an explicitly padded input, sliced (float64)."""
    from mvs_amd import tap_gemm
    g = torch.Generator().manual_seed(sum(n))
    x = torch.randn((2, 3) + n, generator=g, dtype=torch.float64)
    w = torch.randn(4, 3, 3, 3, 3, generator=g, dtype=torch.float64)
    gy = torch.randn((2, 4) + out, generator=g, dtype=torch.float64)
    xa, wa = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    ya = tap_gemm.conv3d_box(xa, wa, 2, pad_lo, out)
    (ya * gy).sum().backward()
    xb, wb = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    # explicit padding: pad_lo before, enough after for every output's window
    after = [max(0, 2 * (o - 1) + 3 - pl - d) for o, pl, d in zip(out, pad_lo, n)]
    xp = torch.nn.functional.pad(xb, (pad_lo[2], after[2], pad_lo[1], after[1], pad_lo[0], after[0]))
    yb = torch.nn.functional.conv3d(xp, wb, stride=2)[:, :, :out[0], :out[1], :out[2]]
    (yb * gy).sum().backward()
    torch.testing.assert_close(ya, yb)
    torch.testing.assert_close(xa.grad, xb.grad)
    torch.testing.assert_close(wa.grad, wb.grad)


@pytest.mark.parametrize("n,crop,out", [((4, 3, 5), (1, 0, 2), (7, 6, 9)), ((3, 4, 4), (0, 1, 1), (8, 7, 9)),
                                        ((5, 2, 3), (2, 1, 0), (6, 5, 8))])
def test_conv_transpose3d_box_matches_sliced(n, crop, out):
    """tap_gemm.conv_transpose3d_box: outputs [crop, crop + out) of the unpadded stride-2 transposed conv
    (zeros past its extent), values and gradients against F.conv_transpose3d, sliced / zero padded."""
    from mvs_amd import tap_gemm
    g = torch.Generator().manual_seed(sum(n) + 7)
    x = torch.randn((2, 4) + n, generator=g, dtype=torch.float64)
    w = torch.randn(4, 3, 3, 3, 3, generator=g, dtype=torch.float64)
    gy = torch.randn((2, 3) + out, generator=g, dtype=torch.float64)
    xa, wa = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    ya = tap_gemm.conv_transpose3d_box(xa, wa, 2, crop, out)
    (ya * gy).sum().backward()
    xb, wb = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    full = torch.nn.functional.conv_transpose3d(xb, wb, stride=2)
    full = torch.nn.functional.pad(full, (0, max(0, crop[2] + out[2] - full.shape[4]), 0,
                                          max(0, crop[1] + out[1] - full.shape[3]), 0,
                                          max(0, crop[0] + out[0] - full.shape[2])))
    yb = full[:, :, crop[0]:crop[0] + out[0], crop[1]:crop[1] + out[1], crop[2]:crop[2] + out[2]]
    (yb * gy).sum().backward()
    torch.testing.assert_close(ya, yb)
    torch.testing.assert_close(xa.grad, xb.grad)
    torch.testing.assert_close(wa.grad, wb.grad)


@pytest.mark.parametrize("cin,cout,k,s,hw", [(3, 8, 3, 1, (13, 17)), (8, 16, 5, 2, (20, 25)), (16, 32, 3, 1, (9, 7)),
                                             (32, 32, 3, 2, (11, 14))])
def test_conv2d_taps_matches_torch(cin, cout, k, s, hw):
    """tap_gemm.conv2d (the encoder / refinement Conv2d under autograd on a HIP device): values and
    gradients against F.conv2d in float64, the reference's kernel / stride / padding k // 2."""
    g = torch.Generator().manual_seed(cin + k)
    x = torch.randn((2, cin) + hw, generator=g, dtype=torch.float64)
    w = torch.randn(cout, cin, k, k, generator=g, dtype=torch.float64)
    xa, wa = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    ya = tap_gemm.conv2d(xa, wa, s, k // 2)
    gy = torch.randn(ya.shape, generator=g, dtype=torch.float64)
    (ya * gy).sum().backward()
    xb, wb = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    yb = F.conv2d(xb, wb, stride=s, padding=k // 2)
    (yb * gy).sum().backward()
    torch.testing.assert_close(ya, yb)
    torch.testing.assert_close(xa.grad, xb.grad)
    torch.testing.assert_close(wa.grad, wb.grad)
