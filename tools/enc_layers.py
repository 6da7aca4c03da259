"""Per-layer GPU time of the 2-D encoder / refinement convolutions (mvs::conv2d, csrc/conv2d_narrow.hip)
at cfg 2 (B=4, V=3, 512 x 640 images; refinement at 128 x 160, B=4), each layer alone (back-to-back
launches, HIP events), plus a checksum of every output so two library builds can be compared bit for bit
(MVS_LIB_PATH selects the library).

Each layer CONV2D_SPLIT_SHAPES covers is also timed on the split-fp16 MFMA kernel (csrc/conv2d_split.hip)
with its deviation from the fp32 kernel.

Usage: python tools/enc_layers.py [--reps N]   (MVS_CONV2D_F16=0: the encoder total on the fp32 kernels)
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
    total = split_total = 0.0
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
        if (cin, cout, k, s) in ops.CONV2D_SPLIT_SHAPES:
            # the split-fp16 MFMA kernel (csrc/conv2d_split.hip) on the same input, its bound words set
            xb = ops.bound_words(1, dev)[0]
            xb[0] = x.abs().max().view(torch.int32)
            fs = lambda: ops.conv2d_split(x, wt, s, xb, None, *bn)
            ys = fs()
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.reps):
                fs()
            e1.record()
            torch.cuda.synchronize()
            mss = e0.elapsed_time(e1) / a.reps
            split_total += (ms - mss) * calls
            by = (x.numel() + ys.numel()) * 4
            print("  split16 %7.4f ms  %6.0f GB/s  max|split - fp32| / max|y| %.2e"
                  % (mss, by / mss / 1e6, ((ys - y).abs().max() / y.abs().max()).item()), flush=True)
            yb = ops.bound_words(1, dev)[0]
            fb = lambda: ops.conv2d_split(x, wt, s, xb, yb, *bn)
            fb()
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.reps):
                fb()
            e1.record()
            torch.cuda.synchronize()
            print("  split16 raising y's bound words %7.4f ms" % (e0.elapsed_time(e1) / a.reps), flush=True)
        yb = ops.bound_words(1, dev)[0]
        fb = lambda: ops.conv2d(x, wt, s, *bn, y_bound=yb)
        fb()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.reps):
            fb()
        e1.record()
        torch.cuda.synchronize()
        print("  fp32 raising y's bound words %7.4f ms" % (e0.elapsed_time(e1) / a.reps), flush=True)
    print("per eval step (x calls): %.4f ms; split16 saves %.4f ms" % (total, split_total), flush=True)
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
    print("feature_encoder (B*V=12, MVS_CONV2D_F16=%s): %.4f ms  sha %s"
          % (os.environ.get("MVS_CONV2D_F16", "1"), e0.elapsed_time(e1) / a.reps,
             hashlib.sha1(f.cpu().numpy().tobytes()).hexdigest()[:12]))


if __name__ == "__main__":
    main()
