"""Debug: where the fused head's y0 / y1 differ from the split path (z, y, x histograms)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for sub in ("deep-multiview-depth-estimation_amd", "oracle", os.path.join("tests", "golden")):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch
from cameras import camera_batch, depth_range
from mvs_amd import ops
from mvs_amd.config import pad_outpad
from mvs_amd import model as M
DEV = torch.device("cuda", 0)
RUNS = [0]
CFGS = [(1, 3, 48, 28, 64), (1, 3, 24, 28, 64), (1, 3, 32, 32, 48), (1, 3, 48, 32, 48)]
if os.environ.get('HEAD_DIFF_BIG'): CFGS = [(4, 3, 192, 128, 160)] * int(os.environ['HEAD_DIFF_BIG'])
for (B, V, D, h, w) in CFGS:
    pad = list(pad_outpad(D, h, w)[0]); n = (D, h, w)
    full = tuple((0, d - 1) for d in n)
    Bq = M._tconv_input_region(full, n, pad); C2 = M._tconv_input_region(Bq, n, pad)
    h1, h2 = M._grow(Bq, n, 1), M._grow(C2, n, 1)
    lo = [max(2 * a - p, 0) for (a, _), p in zip(h2, pad)]
    hi = [min(2 * b - p + 2, d - 1) + 1 for (_, b), p, d in zip(h2, pad, n)]
    if os.environ.get('HEAD_DIFF_FULLBOX'):
        lo, hi = [0, 0, 0], list(n)
    K, R, T = camera_batch(B, V, h, w); d_min, d_int = depth_range(B, d_int=200.0 / D)
    g = torch.Generator().manual_seed(1)
    feat = torch.randn(B * V, 32, h, w, generator=g).to(DEV)
    w0 = (torch.randn(8, 32, 3, 3, 3, generator=g) * 0.1).to(DEV)
    w1 = (torch.randn(16, 32, 3, 3, 3, generator=g) * 0.1).to(DEV)
    org, size = [a for a, _ in h1], [b - a + 1 for a, b in h1]
    with torch.no_grad():
        scv, am = ops.cost_volume_c4_split(feat, K, R, T, d_min, d_int, B, V, 0, D, 25.0)
        y0r = ops.conv3d_k3_split(scv, am, w0)
        y1r = ops.conv_s2_split(scv, am, w1, list(n), org, size, pad)
        y0, y1, box, _ = ops.cost_volume_head(feat, K, R, T, d_min, d_int, B, V, 0, D, 25.0, w0, None, None, None,
                                              w1, None, None, None, pad, org, size, lo, hi)
    torch.cuda.synchronize()
    RUNS[0] += 1
    bad = (y0 != y0r)
    if os.environ.get('HEAD_DIFF_QUIET') and not bad.any() and torch.equal(y1, y1r) and torch.equal(box, scv):
        continue
    print("cfg", (B, V, D, h, w), "y0 bad", int(bad.sum()), "of", bad.numel(), "maxd %.3g" % (y0 - y0r).abs().max().item())
    if bad.any():
        bz = bad.any(4).any(3).any(1)[0].nonzero().flatten().tolist()
        by = bad.any(4).any(2).any(1)[0].nonzero().flatten().tolist()
        bx = bad.any(3).any(2).any(1)[0].nonzero().flatten().tolist()
        print("  z", bz[:60]); print("  y", by[:60]); print("  x", bx[:60])
        nz = bad.nonzero()
        print("  b", sorted(set(nz[:, 0].tolist())))
        tz = (nz[:, 2] // 48).tolist(); ty = (nz[:, 3] // 4).tolist(); tx = (nz[:, 4] // 16).tolist()
        import collections
        tiles = collections.Counter(zip(nz[:, 0].tolist(), tz, ty, tx))
        print("  tiles (b, zc, ty, tx): count", len(tiles), sorted(tiles.items())[:20])
        print("  y0 bad voxels (b,c,z,y,x)", nz[:24].tolist())
        print("  z within chunk", sorted(collections.Counter((nz[:, 2] % 48).tolist()).items())[:48])
        print("  y within tile", sorted(collections.Counter((nz[:, 3] % 4).tolist()).items()))
        bc = bad.any(4).any(3).any(2)[0].nonzero().flatten().tolist(); print("  c", bc)
    bad1 = (y1 != y1r)
    print("  y1 bad", int(bad1.sum()), "of", bad1.numel())
    if bad1.any():
        print("  y1 z", bad1.any(4).any(3).any(2)[0].nonzero().flatten().tolist()[:60])
    sl = (slice(None), slice(None)) + tuple(slice(a, b) for a, b in zip(lo, hi))
    bb = (box != scv[sl]).any(-1)
    print("  box bad", int(bb.sum()), "of", bb.numel())
    if bb.any():
        idx = bb.nonzero()[:8].tolist()
        print("  box bad at (b,q,z,y,x) + origin", [tuple(i[:2]) + tuple(a + o for a, o in zip(i[2:], lo)) for i in idx])
        nzb = bb.nonzero()
        print("  box bad voxels (b,q,z,y,x)", [tuple(i[:2]) + tuple(a + o for a, o in zip(i[2:], lo)) for i in nzb[:40].tolist()])
        print("  box bad z-in-chunk", sorted(set(((nzb[:, 2] + lo[0]) % 48).tolist())), "y", sorted(set((nzb[:, 3] + lo[1]).tolist()))[:20],
              "x", sorted(set((nzb[:, 4] + lo[2]).tolist()))[:20], "q", sorted(set(nzb[:, 1].tolist())))
print("runs", RUNS[0])
