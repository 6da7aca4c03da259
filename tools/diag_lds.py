"""Diagnostic: recover the LDS-path sample values with V=2 and a zero reference view
(cv = s^2/4) and compare them with the v1 warp kernel's sample of the same view."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("deep-multiview-depth-estimation_amd", "oracle", os.path.join("tests", "golden")):
    sys.path.insert(0, os.path.join(REPO, sub))
import numpy as np, torch
from cameras import camera_batch, depth_range, features
from mvs_amd import warp_and_assemble_cost_volume, homography_warping
dev = torch.device("cuda:0")
for ident in (True, False):
    B, V, C, h, w, D = 2, 2, 8, 128, 160, 8
    K3, R3, T3 = camera_batch(B, 3, h, w)
    if ident:
        K = K3[0::3].repeat_interleave(2, 0); R = R3[0::3].repeat_interleave(2, 0); T = T3[0::3].repeat_interleave(2, 0)
    else:
        sel = [0, 1, 3, 4]
        K, R, T = K3[sel], R3[sel], T3[sel]
    d_min, d_int = depth_range(B)
    f = features(B * V, C, h, w, seed=5).to(dev)
    f[0::2] = 0.0
    cv, _, _ = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, f, B, V, d_num=D)
    wp, _, _ = homography_warping(K, R, T, d_min, d_int, f, B, V, d_num=D)
    s = 2 * cv.sqrt()
    ref = wp[1::2].abs()
    d = (s - ref).abs()
    print("ident", ident, "max |s - |warp||", d.max().item(), "frac >1e-6", (d > 1e-6).float().mean().item())
    if d.max() > 1e-6:
        idx = np.unravel_index(int(d.argmax()), d.shape)
        print("  worst at b,c,k,y,x", idx, "lds", s[idx].item(), "warp", ref[idx].item())
        bad = (d > 1e-6).nonzero()
        print("  x mod 16 hist", np.bincount((bad[:, 4] % 16).cpu().numpy(), minlength=16))
        print("  y mod 16 hist", np.bincount((bad[:, 3] % 16).cpu().numpy(), minlength=16))
        print("  k hist", np.bincount(bad[:, 2].cpu().numpy(), minlength=D), "c hist", np.bincount(bad[:, 1].cpu().numpy(), minlength=C))
