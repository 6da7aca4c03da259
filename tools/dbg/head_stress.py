"""Debug: repeatability of the fused head and of the split path it is checked against.

For each geometry: the split path (cost_volume_c4_split -> conv3d_k3_split / conv_s2_split) once as
the reference, then N launches of the head and N more of the split path, each compared with the
reference on every voxel of y0 / y1 / the box.  Prints the count of differing launches per kernel
and, for the first few, where the differing voxels sit (sample, depth chunk, tile, row in tile,
plane within the chunk, channel) -- the head's producer items are (halo voxel, channel quad) of
two planes per step.

Usage: python tools/dbg/head_stress.py [N] [bn]
"""
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for sub in ("deep-multiview-depth-estimation_amd", "oracle", os.path.join("tests", "golden")):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch  # noqa: E402
from cameras import camera_batch, depth_range  # noqa: E402
from mvs_amd import model as M  # noqa: E402
from mvs_amd import ops  # noqa: E402
from mvs_amd.config import pad_outpad  # noqa: E402

DEV = torch.device("cuda", 0)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 50
USE_BN = len(sys.argv) > 2 and sys.argv[2] == "bn"
CFGS = [(1, 2, 20, 24, 40), (1, 3, 16, 29, 41), (2, 3, 16, 32, 48), (1, 3, 48, 28, 64), (4, 3, 192, 128, 160)]
if os.environ.get("HEAD_STRESS_CFGS"):   # e.g. "1,2,20,24,40;1,3,16,29,41"
    CFGS = [tuple(int(v) for v in c.split(",")) for c in os.environ["HEAD_STRESS_CFGS"].split(";")]


def where(bad, tag):
    nz = bad.nonzero()
    if nz.numel() == 0:
        return
    b, c, z, y, x = (nz[:, i] for i in range(5))
    print("   %s: %d voxels; b %s; c %s; z-in-chunk %s; tile (y//4, x//16) %s; y%%4 %s; x%%16 %s" % (
        tag, nz.shape[0], sorted(set(b.tolist()))[:8], sorted(set(c.tolist())),
        sorted(collections.Counter((z % 48).tolist()).items())[:12],
        sorted(collections.Counter(zip((y // 4).tolist(), (x // 16).tolist())).items())[:8],
        sorted(set((y % 4).tolist())), sorted(set((x % 16).tolist()))), flush=True)


for (B, V, D, h, w) in CFGS:
    pad = list(pad_outpad(D, h, w)[0])
    n = (D, h, w)
    full = tuple((0, d - 1) for d in n)
    Bq = M._tconv_input_region(full, n, pad)
    C2 = M._tconv_input_region(Bq, n, pad)
    h1, h2 = M._grow(Bq, n, 1), M._grow(C2, n, 1)
    lo = [max(2 * a - p, 0) for (a, _), p in zip(h2, pad)]
    hi = [min(2 * b - p + 2, d - 1) + 1 for (_, b), p, d in zip(h2, pad, n)]
    K, R, T = camera_batch(B, V, h, w)
    d_min, d_int = depth_range(B, d_int=200.0 / D)
    g = torch.Generator().manual_seed(D + h + w)
    feat = torch.randn(B * V, 32, h, w, generator=g).to(DEV)
    w0 = (torch.randn(8, 32, 3, 3, 3, generator=g) * 0.1).to(DEV)
    w1 = (torch.randn(16, 32, 3, 3, 3, generator=g) * 0.1).to(DEV)
    bn0 = [(torch.rand(8, generator=g) + 0.5).to(DEV), (torch.randn(8, generator=g) * 0.1).to(DEV),
           (torch.randn(8, generator=g) * 0.1).to(DEV)] if USE_BN else [None] * 3
    bn1 = [(torch.rand(16, generator=g) + 0.5).to(DEV), (torch.randn(16, generator=g) * 0.1).to(DEV),
           (torch.randn(16, generator=g) * 0.1).to(DEV)] if USE_BN else [None] * 3
    org, size = [a for a, _ in h1], [b - a + 1 for a, b in h1]
    sl = (slice(None), slice(None)) + tuple(slice(a, b) for a, b in zip(lo, hi))

    def split_path():
        scv, am = ops.cost_volume_c4_split(feat, K, R, T, d_min, d_int, B, V, 0, D, 25.0)
        return (ops.conv3d_k3_split(scv, am, w0, *bn0), ops.conv_s2_split(scv, am, w1, list(n), org, size, pad, *bn1),
                scv[sl])

    def head():
        y0, y1, box, _ = ops.cost_volume_head(feat, K, R, T, d_min, d_int, B, V, 0, D, 25.0, w0, *bn0, w1, *bn1,
                                              pad, org, size, lo, hi)
        return y0, y1, box

    with torch.no_grad():
        ref = split_path()
        ref_full = ops.cost_volume_c4_split(feat, K, R, T, d_min, d_int, B, V, 0, D, 25.0)
        torch.cuda.synchronize()
        counts = {}
        shown = 0
        def split_head():   # the head's consumers fed from the materialised split volume (V = 2 only)
            scv, am = ref_full
            y0, y1 = ops.split_head(scv, am, w0, *bn0, w1, *bn1, pad, org, size)
            return y0, y1, ref[2]
        kinds = [("head", head), ("split", split_path)] + ([("split_head", split_head)] if V == 2 else [])
        for name, fn in kinds:
            nbad = 0
            for it in range(N):
                out = fn()
                torch.cuda.synchronize()
                diff = [not torch.equal(a, b) for a, b in zip(out, ref)]
                if os.environ.get("HEAD_STRESS_BOX_ONLY") and name == "head":   # ablation builds: y0 / y1 not formed
                    diff[0] = diff[1] = False
                if any(diff):
                    nbad += 1
                    if shown < int(os.environ.get("HEAD_STRESS_SHOW", "4")):
                        shown += 1
                        print("  %s launch %d differs: y0 %s y1 %s box %s" % (name, it, *diff), flush=True)
                        if diff[0]:
                            where(out[0] != ref[0], "y0")
                        if diff[2] and os.environ.get("HEAD_STRESS_DETAIL"):
                            # the box holds the ring's split operands: which (quad, plane, y, x) and what was
                            # written instead -- zeros (a lost write), or the value of another voxel / plane
                            bb = (out[2] != ref[2]).any(-1).nonzero()
                            full_ref = ref_full[0]
                            for e in bb[:6].tolist():
                                b_, q, z, y, x = e
                                got = out[2][b_, q, z, y, x].tolist()
                                want = ref[2][b_, q, z, y, x].tolist()
                                zz, yy, xx = z + lo[0], y + lo[1], x + lo[2]
                                hits = (full_ref[b_, q] == out[2][b_, q, z, y, x]).all(-1).nonzero()[:4].tolist()
                                # the wrong half-words alone: hi.y / lo.y = channels 4q+2, 4q+3 (fp16 pairs)
                                wy = out[2][b_, q, z, y, x]
                                h1 = (full_ref[b_, q][..., 1] == wy[1]).nonzero()[:4].tolist()
                                l1 = (full_ref[b_, q][..., 3] == wy[3]).nonzero()[:4].tolist()
                                # low fp16 (channel 4q+2) of hi.y anywhere in the quad plane
                                lo16 = (full_ref[b_, q][..., 1] & 0xFFFF) == (int(wy[1]) & 0xFFFF)
                                print("    box (b%d q%d z%d y%d x%d): head %s ref %s; whole entry in ref at %s; hi.y at %s; lo.y at %s;"
                                      " hi.y low fp16 at %s" % (b_, q, zz, yy, xx, got, want, hits, h1, l1,
                                                               lo16.nonzero()[:6].tolist()), flush=True)
            counts[name] = nbad
    print("cfg", (B, V, D, h, w), "bn" if USE_BN else "raw", "differing launches of %d:" % N, counts, flush=True)
