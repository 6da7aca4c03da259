"""Diagnostic: identical views must give ~zero variance; locate the worst voxel."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("deep-multiview-depth-estimation_amd", "oracle", os.path.join("tests", "golden")):
    sys.path.insert(0, os.path.join(REPO, sub))
import numpy as np, torch
from cameras import camera_batch, depth_range, features
from mvs_amd import warp_and_assemble_cost_volume, homography_warping
dev = torch.device("cuda:0")
B, V, C, h, w, D = 4, 3, 32, 128, 160, 8
K, R, T = camera_batch(B, V, h, w)
d_min, d_int = depth_range(B)
feat = features(B * V, C, h, w, seed=2).to(dev)
same = feat[0::V].repeat_interleave(V, 0).contiguous()
Ks, Rs, Ts = K[0::V].repeat_interleave(V, 0), R[0::V].repeat_interleave(V, 0), T[0::V].repeat_interleave(V, 0)
cvz, _, _ = warp_and_assemble_cost_volume(Ks, Rs, Ts, d_min, d_int, same, B, V, d_num=D)
wz, _, _ = homography_warping(Ks, Rs, Ts, d_min, d_int, same, B, V, d_num=D)
a = cvz.abs()
idx = np.unravel_index(int(a.argmax()), a.shape)
print("max var", a.max().item(), "at b,c,k,y,x", idx, "count>1e-12", int((a > 1e-12).sum()), "of", a.numel())
b, c, k, y, x = idx
print("warp(v1) values views:", [wz[b * V + v, c, k, y, x].item() for v in range(V)])
nz = (a > 1e-12).nonzero()
print("distinct y:", sorted(set(nz[:, 3].tolist()))[:40])
print("distinct x:", sorted(set(nz[:, 4].tolist()))[:40])
print("distinct k:", sorted(set(nz[:, 2].tolist())), "b:", sorted(set(nz[:, 0].tolist())), "c:", sorted(set(nz[:, 1].tolist()))[:8])
