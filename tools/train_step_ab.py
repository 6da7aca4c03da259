"""cfg-2 train.py step (bench.train_step_bench) on the live-region regulariser under autograd
(default) or forward_full (--full: MVS_TRAIN_LIVE=0), with a per-kernel summary from the torch
profiler of one step (--prof).

Usage: python tools/train_step_ab.py [--full] [--steps N] [--prof]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full", action="store_true")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--prof", action="store_true")
    ap.add_argument("--ops", action="store_true", help="with --prof: aten ops grouped by input shape")
    a = ap.parse_args()
    if a.full:
        os.environ["MVS_TRAIN_LIVE"] = "0"
    import bench
    import torch
    dev = torch.device("cuda", 0)
    out = bench.train_step_bench(4, 3, 192, 512, 640, dev, a.steps)
    print(json.dumps(out), flush=True)
    if a.prof:
        from torch.profiler import ProfilerActivity, profile
        net = bench.build_model(192, 512, 640, dev).train()
        opt = torch.optim.Adam(net.parameters, lr=1e-3)
        img, K, R, T, d_min, d_int = bench.make_inputs(4, 3, 512, 640, 0, dev)
        gt = (425.0 + 25.0 * 192 * torch.rand(4, 1, 128, 160)).to(dev)

        def step():
            opt.zero_grad(set_to_none=True)
            ini, ref = net(img, K, R, T, d_min, d_int, 4, 3)
            bench.masked_mae_loss(gt, ini, ref).backward()
            opt.step()
        step()
        torch.cuda.synchronize()
        acts = [ProfilerActivity.CUDA] + ([ProfilerActivity.CPU] if a.ops else [])
        with profile(activities=acts, record_shapes=a.ops) as p:
            step()
            torch.cuda.synchronize()
        print(p.key_averages().table(sort_by="cuda_time_total", row_limit=30, max_name_column_width=70), flush=True)
        if a.ops:
            print(p.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=45,
                                                                  max_name_column_width=40,
                                                                  max_shapes_column_width=110), flush=True)


if __name__ == "__main__":
    main()
