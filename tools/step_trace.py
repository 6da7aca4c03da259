"""Run only the timed end-to-end step (no full-volume leg, no kernel timing, no CPU baseline), so a
rocprofv3 --kernel-trace --stats run of this script shows where one bench step's GPU time goes.

Usage: python tools/step_trace.py [--mode eval|train] [--steps N] [--batch B] [--planes D]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=("eval", "train", "grad"), default="eval")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--planes", type=int, default=192)
    ap.add_argument("--views", type=int, default=3)
    ap.add_argument("--arithmetic", choices=("fp32", "split_f16"), default="fp32")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B, V, D, H, W = a.batch, a.views, a.planes, 512, 640
    net = bench.build_model(D, H, W, dev, arithmetic=a.arithmetic)
    if a.mode != "eval":
        net.train()
    inputs = bench.make_inputs(B, V, H, W, 0, dev)
    if a.mode == "grad":
        def step():
            ini, ref = net(*inputs, B, V)
            (ini.mean() + ref.mean()).backward()
        ctx = torch.enable_grad
    else:
        step = lambda: net(*inputs, B, V)
        ctx = torch.no_grad
    with ctx():
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
    print("%s step: %.2f ms" % (a.mode, 1000.0 * (time.perf_counter() - t) / a.steps), flush=True)


if __name__ == "__main__":
    main()
