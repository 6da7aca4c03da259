"""N fp32 eval steps of the headline workload (cfg 2: B=4, V=3, 640x512, D=192, BN eval, MVSNet.forward
under no_grad), nothing else -- the program the per-leg rocprof stats and PMC passes of the eval step run.

Usage: python tools/eval_steps.py [--steps N] [--arithmetic fp32|split_f16]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--arithmetic", default="fp32")
    a = ap.parse_args()
    import bench
    import torch
    dev = torch.device("cuda", 0)
    net = bench.build_model(192, 512, 640, dev, arithmetic=a.arithmetic)
    img, K, R, T, d_min, d_int = bench.make_inputs(4, 3, 512, 640, 0, dev)
    with torch.no_grad():
        for _ in range(2 + a.steps):
            net(img, K, R, T, d_min, d_int, 4, 3)
    torch.cuda.synchronize()
    print("ok", flush=True)


if __name__ == "__main__":
    main()
