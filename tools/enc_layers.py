"""Per-layer GPU time of the 2-D encoder / refinement convolutions (mvs::conv2d, csrc/conv2d_narrow.hip)
at cfg 2 (B=4, V=3, 512 x 640 images; refinement at 128 x 160, B=4), each layer alone (back-to-back
launches, HIP events), plus a checksum of every output so two library builds can be compared bit for bit
(MVS_LIB_PATH selects the library).

Usage: python tools/enc_layers.py [--reps N]
"""
import argparse
import hashlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402
from mvs_amd import ops  # noqa: E402

# (c_in, c_out, k, stride, n, h, w, calls per eval step)
LAYERS = [(3, 8, 3, 1, 12, 512, 640, 1), (8, 8, 3, 1, 12, 512, 640, 1), (8, 16, 5, 2, 12, 512, 640, 1),
          (16, 16, 3, 1, 12, 256, 320, 2), (16, 32, 5, 2, 12, 256, 320, 1), (32, 32, 3, 1, 12, 128, 160, 2),
          (4, 32, 3, 1, 4, 128, 160, 1), (32, 32, 3, 1, 4, 128, 160, 2), (32, 1, 3, 1, 4, 128, 160, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(7)
    total = 0.0
    for cin, cout, k, s, n, h, w, calls in LAYERS:
        x = torch.randn(n, cin, h, w, generator=g).to(dev)
        wt = (torch.randn(cout, cin, k, k, generator=g) * 0.2).to(dev)
        bn = [(torch.rand(cout, generator=g) + 0.5).to(dev), (torch.randn(cout, generator=g) * 0.1).to(dev),
              (torch.randn(cout, generator=g) * 0.1).to(dev)] if cout > 1 else [None, None, None]
        fn = lambda: ops.conv2d(x, wt, s, *bn)
        y = fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        total += ms * calls
        ho, wo = y.shape[2], y.shape[3]
        fl = 2.0 * n * ho * wo * cout * cin * k * k
        digest = hashlib.sha1(y.cpu().numpy().tobytes()).hexdigest()[:12]
        print("conv2d %2d->%-2d k%d s%d n%-2d %3dx%-3d  %7.4f ms  %6.1f TF/s  x%d  sha %s"
              % (cin, cout, k, s, n, h, w, ms, fl / ms / 1e9, calls, digest), flush=True)
    print("per eval step (x calls): %.4f ms" % total, flush=True)
    dev_ = dev
    B, V, D, H, W = 4, 3, 192, 512, 640
    net = bench.build_model(D, H, W, dev_)
    img = bench.make_inputs(B, V, H, W, 0, dev_)[0]
    with torch.no_grad():
        f = net.feature_encoder(img)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            net.feature_encoder(img)
        e1.record()
        torch.cuda.synchronize()
    print("feature_encoder (B*V=12): %.4f ms  sha %s" % (e0.elapsed_time(e1) / a.reps,
                                                          hashlib.sha1(f.cpu().numpy().tobytes()).hexdigest()[:12]))


if __name__ == "__main__":
    main()
