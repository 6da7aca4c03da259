"""Debug: GPU time of the cost-volume head variants at the bench geometry (B 4, V 3, D 192, 128 x 160).

  split volume   cost_volume_c4_split (materialised, 128 B / voxel)
  conv_0_0       conv3d_k3_split on it;  conv_1_0  conv_s2_split on halo(B)
  split head     ops.split_head: both convolutions in one pass over the split volume
  fused head     ops.cost_volume_head: variance formed on chip, box stored
Median of N launches each (HIP events on the current stream).
Usage: python tools/dbg/head_time.py [N]
"""
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
N = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B, V, D, h, w = (int(v) for v in os.environ.get("HEAD_TIME_CFG", "4,3,192,128,160").split(","))
pad = list(pad_outpad(D, h, w)[0])
n = (D, h, w)
full = tuple((0, d - 1) for d in n)
Bq = M._tconv_input_region(full, n, pad)
C2 = M._tconv_input_region(Bq, n, pad)
h1, h2 = M._grow(Bq, n, 1), M._grow(C2, n, 1)
lo = [max(2 * a - p, 0) for (a, _), p in zip(h2, pad)]
hi = [min(2 * b - p + 2, d - 1) + 1 for (_, b), p, d in zip(h2, pad, n)]
org, size = [a for a, _ in h1], [b - a + 1 for a, b in h1]
K, R, T = camera_batch(B, V, h, w)
d_min, d_int = depth_range(B, d_int=200.0 / D)
g = torch.Generator().manual_seed(1)
feat = torch.randn(B * V, 32, h, w, generator=g).to(DEV)
w0 = (torch.randn(8, 32, 3, 3, 3, generator=g) * 0.1).to(DEV)
w1 = (torch.randn(16, 32, 3, 3, 3, generator=g) * 0.1).to(DEV)
bn0 = [(torch.rand(8, generator=g) + 0.5).to(DEV), (torch.randn(8, generator=g) * 0.1).to(DEV),
       (torch.randn(8, generator=g) * 0.1).to(DEV)]
bn1 = [(torch.rand(16, generator=g) + 0.5).to(DEV), (torch.randn(16, generator=g) * 0.1).to(DEV),
       (torch.randn(16, generator=g) * 0.1).to(DEV)]


def timed(fn):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(N):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


with torch.no_grad():
    scv, am = ops.cost_volume_c4_split(feat, K, R, T, d_min, d_int, B, V, 0, D, 25.0)
    res = {
        "split volume": timed(lambda: ops.cost_volume_c4_split(feat, K, R, T, d_min, d_int, B, V, 0, D, 25.0)),
        "conv_0_0 split": timed(lambda: ops.conv3d_k3_split(scv, am, w0, *bn0)),
        "conv_1_0 split": timed(lambda: ops.conv_s2_split(scv, am, w1, list(n), org, size, pad, *bn1)),
        "split head": timed(lambda: ops.split_head(scv, am, w0, *bn0, w1, *bn1, pad, org, size)),
    }
    if V in (2, 3):
        res["fused head"] = timed(lambda: ops.cost_volume_head(feat, K, R, T, d_min, d_int, B, V, 0, D, 25.0, w0, *bn0,
                                                               w1, *bn1, pad, org, size, lo, hi))
print("cfg", (B, V, D, h, w), {k: round(v, 3) for k, v in res.items()}, flush=True)
print("split path (volume + 2 convs) %.3f ms; volume + split head %.3f ms" % (
    res["split volume"] + res["conv_0_0 split"] + res["conv_1_0 split"], res["split volume"] + res["split head"]))
