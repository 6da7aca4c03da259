"""Per-layer forward + backward time of the regulariser's convolutions in the cfg-2 train step on the
live-region path under autograd (CostVolumeReg.forward_live_train), per-tap rocBLAS GEMMs
(tap_gemm) against MIOpen (F.conv3d / F.conv_transpose3d): the calls of one step are recorded, then
each is timed alone (x and w requiring grad, a random output gradient).

Usage: python tools/train_layers.py [--reps N]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from mvs_amd import model as M  # noqa: E402
from mvs_amd import tap_gemm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    calls = []
    o_c, o_t, o_tc = M._region_conv3d, M._region_conv_transpose3d, M._train_conv

    def rc(x, w, s, p):
        calls.append(("conv", tuple(x.shape), tuple(w.shape), s, p))
        return o_c(x, w, s, p)

    def rt(x, w, s):
        calls.append(("tconv", tuple(x.shape), tuple(w.shape), s, 0))
        return o_t(x, w, s)

    def tc(m, x):
        calls.append(("conv", tuple(x.shape), tuple(m.weight.shape), m.stride, m.padding))
        return o_tc(m, x)
    M._region_conv3d, M._region_conv_transpose3d, M._train_conv = rc, rt, tc
    net = bench.build_model(192, 512, 640, dev).train()
    img, K, R, T, d_min, d_int = bench.make_inputs(4, 3, 512, 640, 0, dev)
    ini, ref = net(img, K, R, T, d_min, d_int, 4, 3)
    (ini.sum() + ref.sum()).backward()
    M._region_conv3d, M._region_conv_transpose3d, M._train_conv = o_c, o_t, o_tc
    del net, ini, ref
    torch.cuda.empty_cache()
    print("%d regulariser conv calls" % len(calls), flush=True)
    tot = {"taps": 0.0, "miopen": 0.0}
    for kind, xs, ws, s, p in calls:
        x = torch.randn(xs, device=dev, requires_grad=True)
        w = (torch.randn(ws, device=dev) * 0.05).requires_grad_(True)
        fns = {"taps": (lambda: tap_gemm.conv3d(x, w, s, p)) if kind == "conv" else
                       (lambda: tap_gemm.conv_transpose3d(x, w, s)),
               "miopen": (lambda: F.conv3d(x, w, stride=s, padding=p)) if kind == "conv" else
                         (lambda: F.conv_transpose3d(x, w, stride=s))}
        row = []
        for name, fn in fns.items():
            y = fn()
            gy = torch.randn_like(y)
            y.backward(gy)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                x.grad = w.grad = None
                fn().backward(gy)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            tot[name] += ms
            row.append("%s %8.2f ms" % (name, ms))
        print("%-6s x%-28s w%-20s s%s p%s  %s" % (kind, xs, ws, s, p, "  ".join(row)), flush=True)
        del x, w
        torch.cuda.empty_cache()
    print("total: taps %.1f ms, miopen %.1f ms" % (tot["taps"], tot["miopen"]), flush=True)


if __name__ == "__main__":
    main()
