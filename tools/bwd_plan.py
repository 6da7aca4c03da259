"""CPU model of the backward kernel's LDS pass planner (csrc/cost_volume_bwd.hip).

Per (sample, 32x8 tile, 32-plane group): the per-(plane, source view) tap boxes (float64 sampling
law, tests/footprint.py), the view subsets and the passes of consecutive planes whose union fits
the slot budget, as the kernel plans them.  Prints passes per workgroup, flushed slots and the
planes that overflow to the global-atomic path for each budget.

Usage: python tools/bwd_plan.py B V h w D slots[,slots...]    e.g. 4 3 128 160 192 921,1228
"""
import os
import sys

import numpy as np  # noqa: F401

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
from footprint import tap_corners
from cameras import camera_batch, depth_range
B, V, h, w, D = [int(x) for x in sys.argv[1:6]]
budgets = [int(x) for x in sys.argv[6].split(',')]
K, R, T = (x.double().numpy() for x in camera_batch(B, V, h, w))
d_min, d_int = depth_range(B)
x0, y0, ok = tap_corners(K, R, T, d_min.numpy(), d_int.numpy(), B, V, h, w, list(range(D)))
NS = V - 1; TW, TH, KPG = 32, 8, 32
def area(bx): return 0 if bx is None else (bx[2]-bx[0]+1)*(bx[3]-bx[1]+1)
def union(a, b):
    if a is None: return b
    if b is None: return a
    return (min(a[0],b[0]), min(a[1],b[1]), max(a[2],b[2]), max(a[3],b[3]))
boxes = {}
for b in range(B):
  for ty in range(0, h, TH):
    for tx in range(0, w, TW):
      for s in range(NS):
        for k in range(D):
          m = ok[b, s, k, ty:ty+TH, tx:tx+TW]
          if not m.any(): boxes[b,ty,tx,s,k] = None; continue
          xx = x0[b, s, k, ty:ty+TH, tx:tx+TW][m]; yy = y0[b, s, k, ty:ty+TH, tx:tx+TW][m]
          boxes[b,ty,tx,s,k] = (max(xx.min(), -1), max(yy.min(), -1), min(xx.max()+1, w), min(yy.max()+1, h))
for S in budgets:
  passes = flush = glob_planes = wg = 0; subsets = 0
  for b in range(B):
    for ty in range(0, h, TH):
      for tx in range(0, w, TW):
        for g0 in range(0, D, KPG):
          wg += 1
          npl = min(KPG, D - g0)
          amax = [max(area(boxes[b,ty,tx,s,g0+p]) for p in range(npl)) for s in range(NS)]
          s0 = 0
          while s0 < NS:
            s1 = s0 + 1; sa = amax[s0]
            while s1 < NS and sa + amax[s1] <= S: sa += amax[s1]; s1 += 1
            subsets += 1
            kp = 0
            while kp < npl:
              ub = [boxes[b,ty,tx,s,g0+kp] if s0 <= s < s1 else None for s in range(NS)]
              a = sum(area(x) for x in ub); ke = kp + 1
              if a <= S:
                while ke < npl:
                  nb = [union(ub[s], boxes[b,ty,tx,s,g0+ke]) if s0 <= s < s1 else ub[s] for s in range(NS)]
                  na = sum(area(x) for x in nb)
                  if na > S: break
                  ub = nb; a = na; ke += 1
              passes += 1
              if a <= S: flush += a
              else: glob_planes += ke - kp
              kp = ke
            s0 = s1
  print(f"slots {S}: WGs {wg} subsets/WG {subsets/wg:.2f} passes/WG {passes/wg:.2f} flush slots/WG {flush/wg:.0f} planes on global path {glob_planes} ({glob_planes/(wg*KPG)*100:.2f}% of WG-planes)")
