"""The tap-GEMM conv reference (tests/tap_conv.py) against PyTorch's CPU convolutions: the shapes
the regulariser uses (stride 1 padding 1; stride 2 with padding n//2 + 1; transposed stride 2 with
output padding), odd and even extents."""
import pytest
import torch
import torch.nn.functional as F

from tap_conv import conv3d_taps, conv_transpose3d_taps, tap_convs


@pytest.mark.parametrize("n", [(5, 6, 7), (8, 9, 10)])
@pytest.mark.parametrize("stride,pad", [(1, 1), (2, None), (2, 0)])
def test_conv3d_taps_matches_torch(n, stride, pad):
    g = torch.Generator().manual_seed(sum(n) + stride)
    x = torch.randn(2, 5, *n, generator=g, dtype=torch.float64)
    w = torch.randn(3, 5, 3, 3, 3, generator=g, dtype=torch.float64)
    p = tuple(d // 2 + 1 for d in n) if pad is None else pad
    torch.testing.assert_close(conv3d_taps(x, w, stride=stride, padding=p),
                               F.conv3d(x, w, stride=stride, padding=p), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("n", [(5, 6, 7), (8, 9, 10)])
def test_conv_transpose3d_taps_matches_torch(n):
    g = torch.Generator().manual_seed(sum(n))
    x = torch.randn(2, 4, *n, generator=g, dtype=torch.float64)
    w = torch.randn(4, 3, 3, 3, 3, generator=g, dtype=torch.float64)
    p = tuple(d // 2 + 1 for d in n)
    op = tuple((d + 1) % 2 for d in n)
    torch.testing.assert_close(conv_transpose3d_taps(x, w, stride=2, padding=p, output_padding=op),
                               F.conv_transpose3d(x, w, stride=2, padding=p, output_padding=op),
                               rtol=1e-12, atol=1e-12)


def test_tap_convs_routes_modules():
    conv = torch.nn.Conv3d(2, 3, 3, padding=1, bias=False).double()
    x = torch.randn(1, 2, 4, 5, 6, dtype=torch.float64)
    ref = conv(x)
    with tap_convs():
        assert F.conv3d is conv3d_taps
        out = conv(x)
    assert F.conv3d is not conv3d_taps
    torch.testing.assert_close(out, ref, rtol=1e-12, atol=1e-12)
