"""Time the fused cost-volume op's backward (mvs::cost_volume_backward: recompute + fixed-point scatter
into grad_feat) beside its forward, through torch autograd, at BASELINE configs.

Usage: python tools/bwd_bench.py [cfg ...]   (cfg in 1, 2, 3; default all)
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402,F401
import torch  # noqa: E402
from cameras import camera_batch, depth_range  # noqa: E402
from mvs_amd import warp_and_assemble_cost_volume  # noqa: E402

CFGS = {"1": (1, 3, 128, 160, 48), "2": (4, 3, 128, 160, 192), "3": (8, 5, 128, 160, 192)}


def main():
    dev = torch.device("cuda", 0)
    for name in (sys.argv[1:] or list(CFGS)):
        B, V, h, w, D = CFGS[name]
        K, R, T = camera_batch(B, V, h, w)
        d_min, d_int = depth_range(B)
        g = torch.Generator().manual_seed(3)
        feat = torch.randn(B * V, 32, h, w, generator=g).to(dev).requires_grad_(True)
        gcv = torch.randn(B, 32, D, h, w, generator=g).to(dev)

        def fwd():
            return warp_and_assemble_cost_volume(K, R, T, d_min, d_int, feat, B, V, d_num=D)[0]

        def timed(n=5):
            cv = fwd()
            cv.backward(gcv)
            torch.cuda.synchronize()
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            tf = tb = 0.0
            for _ in range(n):
                feat.grad = None
                e[0].record()
                cv = fwd()
                e[1].record()
                cv.backward(gcv)
                e[2].record()
                torch.cuda.synchronize()
                tf += e[0].elapsed_time(e[1])
                tb += e[1].elapsed_time(e[2])
            return tf / n, tb / n

        tf, tb = timed()
        torch.use_deterministic_algorithms(True)   # MVS_BWD_DETERMINISTIC (fixed-point backward)
        try:
            _, td = timed()
        finally:
            torch.use_deterministic_algorithms(False)
        print(json.dumps({"cfg": name, "B": B, "V": V, "D": D, "fwd_ms": round(tf, 3),
                          "bwd_ms": round(tb, 3), "det_bwd_ms": round(td, 3)}), flush=True)


if __name__ == "__main__":
    main()
