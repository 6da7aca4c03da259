"""One cfg-2 train.py step (bench.train_step_bench, 1 timed step after the first) for a rocprofv3
kernel trace of the training step alone: python tools/train_step_prof.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402

if __name__ == "__main__":
    # MVS_TRAIN_MARK=1: a torch.cumprod launch on a 1-element tensor at every torch.cuda.synchronize;
    # the timed step is the kernels between the last two marks (tools/trace_between_marks.py)
    if os.environ.get("MVS_TRAIN_MARK"):
        dev = torch.device("cuda", 0)
        orig_sync = torch.cuda.synchronize

        def sync(*a, **k):
            orig_sync(*a, **k)
            torch.cumprod(torch.ones(1, device=dev), 0)
            orig_sync()
        torch.cuda.synchronize = sync
    r = bench.train_step_bench(4, 3, 192, 512, 640, torch.device("cuda", 0), 1)
    print({k: r[k] for k in ("ms_per_step", "first_step_ms", "loss", "peak_mem_GB")}, flush=True)
