"""CPU model of the fused forward kernel's per-workgroup LDS footprint (test helper).

Mirrors the staging decision of ``cost_volume_staged_kernel`` (csrc/cost_volume_fwd.hip): a
256-thread workgroup owns a 32 x 8 pixel tile of one sample and a group of ``pg`` planes; per source
view the bounding box of the valid nw tap corners over the group is staged in LDS with rows padded
to 16 slots (retried unpadded when over budget), plus a zero area; a group still over the budget
takes the global-gather fallback.  Tap corners follow the analytic float64 sampling law
(``oracle/mvs_oracle.py::cost_volume_fp64``), so the model matches the kernel up to fp32 rounding
at corner boundaries -- good enough to pick workloads and planes that exercise each path.
"""
import numpy as np

TILE_W, TILE_H = 32, 8


def group_planes(n_views):
    return 8 if n_views <= 3 else (4 if n_views <= 5 else 2)


def lds_slots(n_views):
    return 2560 if n_views <= 3 else (3072 if n_views <= 5 else 4096)


def launch_group_planes(B, n_views, h, w, d_count, min_workgroups=1024):
    """The plane-group size the launcher picks (halved until the grid is large enough)."""
    pg = group_planes(n_views)
    tiles = -(-w // TILE_W) * -(-h // TILE_H)
    while pg > 1 and B * tiles * -(-d_count // pg) < min_workgroups:
        pg //= 2
    return pg


def tap_corners(K, R, T, d_min, d_int, B, V, h, w, planes, d_scale=25.0):
    """nw tap corners of every (sample, source view, plane, pixel): (x0, y0, valid) int arrays of
    shape [B, V-1, len(planes), h, w]."""
    K = np.asarray(K, np.float64)
    R = np.asarray(R, np.float64)
    T = np.asarray(T, np.float64).reshape(-1, 3, 1)
    d_min = np.asarray(d_min, np.float64).reshape(-1)
    d_int = np.asarray(d_int, np.float64).reshape(-1)
    ys, xs = np.meshgrid(np.arange(h, dtype=np.float64), np.arange(w, dtype=np.float64), indexing="ij")
    pix = np.stack([xs.ravel(), ys.ravel(), np.ones(h * w)])
    shape = (B, V - 1, len(planes), h, w)
    x0 = np.zeros(shape, np.int64)
    y0 = np.zeros(shape, np.int64)
    ok = np.zeros(shape, bool)
    for b in range(B):
        r = b * V
        C_r = -R[r].T @ T[r]
        n_r = R[r][:, 2:3].T
        for s in range(1, V):
            i = r + s
            C_i = -R[i].T @ T[i]
            for j, k in enumerate(planes):
                d = d_min[i % B] + d_scale * d_int[i % B] * k
                H = K[i] @ R[i] @ (np.eye(3) - (C_i - C_r) @ n_r / d) @ R[r].T @ np.linalg.inv(K[r])
                src = np.linalg.inv(H) @ pix
                with np.errstate(divide="ignore", invalid="ignore"):
                    ix = (src[0] / src[2]) * w / (w - 1) - 0.5
                    iy = (src[1] / src[2]) * h / (h - 1) - 0.5
                good = (ix >= -1) & (ix < w) & (iy >= -1) & (iy < h)
                x0[b, s - 1, j] = np.where(good, np.floor(np.where(good, ix, 0)), 0).reshape(h, w)
                y0[b, s - 1, j] = np.where(good, np.floor(np.where(good, iy, 0)), 0).reshape(h, w)
                ok[b, s - 1, j] = good.reshape(h, w)
    return x0, y0, ok


def group_slots(x0, y0, ok, padded=True):
    """LDS slots one workgroup needs for the corners of its (views, planes, tile pixels)."""
    total, zero = 0, 0
    for s in range(x0.shape[0]):
        m = ok[s]
        if not m.any():
            continue
        xx, yy = x0[s][m], y0[s][m]
        rw = int(xx.max() - xx.min() + 2)
        rh = int(yy.max() - yy.min() + 2)
        rp = (rw + 15) & ~15 if padded else rw
        zero = max(zero, rp + 2)
        total += rp * rh
    return total + ((zero + 15) & ~15)


def fallback_map(K, R, T, d_min, d_int, B, V, h, w, d_begin, d_count, pg=None):
    """Boolean [B, groups, tiles_y, tiles_x]: True where the workgroup takes the global-gather
    fallback (over budget even with unpadded rows)."""
    pg = pg or launch_group_planes(B, V, h, w, d_count)
    planes = list(range(d_begin, d_begin + d_count))
    x0, y0, ok = tap_corners(K, R, T, d_min, d_int, B, V, h, w, planes)
    budget = lds_slots(V) - 1
    groups = -(-d_count // pg)
    ty_n, tx_n = -(-h // TILE_H), -(-w // TILE_W)
    out = np.zeros((B, groups, ty_n, tx_n), bool)
    for b in range(B):
        for g in range(groups):
            ps = slice(g * pg, min((g + 1) * pg, d_count))
            for ty in range(ty_n):
                for tx in range(tx_n):
                    sl = (b, slice(None), ps, slice(ty * TILE_H, (ty + 1) * TILE_H),
                          slice(tx * TILE_W, (tx + 1) * TILE_W))
                    a, c, m = x0[sl], y0[sl], ok[sl]
                    if group_slots(a, c, m) <= budget:
                        continue
                    out[b, g, ty, tx] = group_slots(a, c, m, padded=False) > budget
    return out, pg
