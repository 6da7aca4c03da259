"""CPU model of the staged kernel's per-workgroup LDS footprint (cost_volume_staged_kernel).

For each (sample, 32x8 tile, plane group) it computes, per source view, the bounding box of the
valid nw tap corners over the group's planes, the padded slot count (rows padded to 16 slots, plus
the zero area) and whether it fits the LDS budget.  Geometry follows the analytic sampling law
(oracle/mvs_oracle.py::cost_volume_fp64), so it matches the kernel up to fp32 rounding at corner
boundaries.

Usage: python tools/footprint_stats.py [cfg] [planes_per_group] [slots]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
from cameras import camera_batch  # noqa: E402

CFGS = {"2": (4, 3, 128, 160, 192), "3": (8, 5, 128, 160, 192), "5": (1, 3, 296, 400, 256)}
TW, TH = 32, 8


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "2"
    B, V, h, w, D = CFGS[cfg]
    kpg = int(sys.argv[2]) if len(sys.argv) > 2 else (8 if V <= 3 else 4)
    budget = int(sys.argv[3]) if len(sys.argv) > 3 else (2560 if V <= 3 else (3072 if V <= 5 else 4096))
    K, R, T = (x.double().numpy() for x in camera_batch(B, V, h, w))
    T = T.reshape(-1, 3, 1)
    ys, xs = np.meshgrid(np.arange(h, dtype=np.float64), np.arange(w, dtype=np.float64), indexing="ij")
    pix = np.stack([xs.ravel(), ys.ravel(), np.ones(h * w)])
    slots_all, fits = [], 0
    n_items = 0
    for b in range(B):
        r = b * V
        C_r = -R[r].T @ T[r]
        n_r = R[r][:, 2:3].T
        # nw corners per (view, plane, pixel); invalid = all taps outside
        x0 = np.zeros((V - 1, D, h, w), np.int64)
        y0 = np.zeros((V - 1, D, h, w), np.int64)
        ok = np.zeros((V - 1, D, h, w), bool)
        for s in range(1, V):
            i = r + s
            C_i = -R[i].T @ T[i]
            for k in range(D):
                d = 425.0 + 25.0 * k
                H = K[i] @ R[i] @ (np.eye(3) - (C_i - C_r) @ n_r / d) @ R[r].T @ np.linalg.inv(K[r])
                src = np.linalg.inv(H) @ pix
                ix = (src[0] / src[2]) * w / (w - 1) - 0.5
                iy = (src[1] / src[2]) * h / (h - 1) - 0.5
                fx, fy = np.floor(ix), np.floor(iy)
                good = (fx >= -1) & (fx <= w - 1) & (fy >= -1) & (fy <= h - 1)
                x0[s - 1, k] = np.where(good, fx, 0).reshape(h, w)
                y0[s - 1, k] = np.where(good, fy, 0).reshape(h, w)
                ok[s - 1, k] = good.reshape(h, w)
        for ty in range(0, h, TH):
            for tx in range(0, w, TW):
                for k0 in range(0, D, kpg):
                    sl = (slice(None), slice(k0, k0 + kpg), slice(ty, ty + TH), slice(tx, tx + TW))
                    total, zero = 0, 0
                    for s in range(V - 1):
                        m = ok[s][sl[1:]]
                        if not m.any():
                            continue
                        xx, yy = x0[s][sl[1:]][m], y0[s][sl[1:]][m]
                        rw = xx.max() - xx.min() + 2
                        rh = yy.max() - yy.min() + 2
                        rp = rw if os.environ.get("NOPAD") else (rw + 15) & ~15
                        zero = max(zero, rp + 2)
                        total += rp * rh
                    total += (zero + 15) & ~15
                    slots_all.append(total)
                    fits += total <= budget
                    n_items += 1
    a = np.array(slots_all)
    print("cfg %s V=%d kpg=%d budget=%d: items %d, fit %.4f, slots mean %.0f p50 %.0f p90 %.0f p99 %.0f max %d"
          % (cfg, V, kpg, budget, n_items, fits / n_items, a.mean(), np.median(a), np.percentile(a, 90),
             np.percentile(a, 99), a.max()))


if __name__ == "__main__":
    main()
