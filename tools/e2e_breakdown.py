"""Where one end-to-end MVSNet.forward step goes (cfg 2, eval BN), by torch op, on the GPU; and
the step time with the regulariser in channels-last-3d layout.

Usage: python tools/e2e_breakdown.py
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402


def step_ms(fn, n=5):
    with torch.no_grad():
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
    return 1000.0 * (time.perf_counter() - t) / n


def main():
    dev = torch.device("cuda", 0)
    B, V, D, H, W = 4, 3, 192, 512, 640
    net = bench.build_model(D, H, W, dev)
    inputs = bench.make_inputs(B, V, H, W, 0, dev)
    step = lambda: net(*inputs, B, V)
    print("live step ms %.2f" % step_ms(step), flush=True)
    from torch.profiler import profile, ProfilerActivity
    with torch.no_grad(), profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25, max_name_column_width=60),
          flush=True)
    reg = net.cost_volume_reg
    reg.to(memory_format=torch.channels_last_3d)
    orig = reg.forward_live

    def cl_forward(cv):
        return orig(cv.contiguous(memory_format=torch.channels_last_3d))
    reg.forward_live = cl_forward
    print("live step ms, regulariser channels_last_3d %.2f" % step_ms(step), flush=True)


if __name__ == "__main__":
    main()
