"""Time the fused cost-volume op (HIP events on the launch stream) over BASELINE configs.

Usage: python tools/kernel_bench.py [cfg ...]   (cfg in 2, 3, 4, 5; default all)
Prints one JSON line per config: main-kernel ms per launch, whole-op ms, algorithmic GB/s, fraction of 8 TB/s.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402  (reuses time_kernel / camera setup)
import torch  # noqa: E402

CFGS = {  # name: (B, V, h, w, D_total, d_count)
    "2": (4, 3, 128, 160, 192, 192),
    "3": (8, 5, 128, 160, 192, 192),
    "4": (1, 3, 128, 160, 256, 32),
    "5": (1, 3, 296, 400, 256, 256),
}


def main():
    dev = torch.device("cuda", 0)
    for name in (sys.argv[1:] or list(CFGS)):
        B, V, h, w, D, dc = CFGS[name]
        C = int(os.environ.get("MVS_BENCH_C", "32"))   # channel-count sweeps (set-up vs per-chunk cost)
        bf16 = os.environ.get("MVS_BENCH_BF16") == "1"
        quads = os.environ.get("MVS_BENCH_C4") == "1"   # channel-quad store (inference feed)
        store = "c4" if quads and not bf16 else "ncdhw"   # (fp32 channel quads: the inference step's store)
        ms, op_ms, alg = bench.time_kernel(B, V, C, h, w, D, dev, 20, 0, dc, bf16=bf16, quads=quads, store=store)
        ms = op_ms if ms is None else ms
        gbs = alg / (ms * 1e-3) / 1e9
        print(json.dumps({"cfg": name, "C": C, "B": B, "V": V, "hw": [h, w], "D": dc, "ms": round(ms, 4),
                          "op_ms": round(op_ms, 4),
                          "alg_GB": round(alg / 1e9, 4), "GBps": round(gbs, 1),
                          "frac_8TBps": round(gbs / 8000.0, 4), "c4": quads}), flush=True)


if __name__ == "__main__":
    main()
