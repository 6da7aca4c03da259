"""Time mvs::conv3d_k3 (conv_0_0 32->8 and conv_out 8->1) at the cfg2 regulariser shape, NCDHW and
channel-quad inputs, with HIP events.  MVS_LIB_PATH selects the library build (A/B experiments).

Usage: python tools/conv_bench.py [iters]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deep-multiview-depth-estimation_amd"))
import torch  # noqa: E402

from mvs_amd.ops import conv3d_k3  # noqa: E402


def timed(fn, iters):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    B, D, H, W = 4, 192, 128, 160
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, 32, D, H, W, device=dev, generator=g)
    x4 = x.reshape(B, 8, 4, D, H, W).permute(0, 1, 3, 4, 5, 2).contiguous()
    w8 = torch.randn(8, 32, 3, 3, 3, device=dev, generator=g) * 0.1
    y8 = torch.randn(B, 8, D, H, W, device=dev, generator=g)
    w1 = torch.randn(1, 8, 3, 3, 3, device=dev, generator=g) * 0.1
    sc, sh, mu = (torch.rand(8, device=dev, generator=g) + 0.5 for _ in range(3))
    flop = 2.0 * B * D * H * W * 27
    with torch.no_grad():
        ref = conv3d_k3(x, w8, sc, sh, mu)
        assert torch.equal(conv3d_k3(x4, w8, sc, sh, mu, in_c4=True), ref)
        for name, fn, f in (("conv_0_0 ncdhw", lambda: conv3d_k3(x, w8, sc, sh, mu), flop * 256),
                            ("conv_0_0 c4", lambda: conv3d_k3(x4, w8, sc, sh, mu, in_c4=True), flop * 256),
                            ("conv_out", lambda: conv3d_k3(y8, w1), flop * 8)):
            ms = timed(fn, iters)
            print("%-16s %.3f ms  %.1f TFLOP/s" % (name, ms, f / ms / 1e9), flush=True)


if __name__ == "__main__":
    main()
