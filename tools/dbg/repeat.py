"""Repeatability stress (hazard audit): every kernel of the eval step and the deterministic backward
run many times on the same inputs must give bit-identical results -- a register or memory race that
lets a wave read data before it lands shows up as a run that differs.

  eval step (cfg 2, B=4): MVSNet.forward N times; the regulariser's probability volume (forward hook)
      and both depth maps compared bitwise with the first run
  backward (cfg 2): mvs::cost_volume_backward(deterministic=True) M times, compared bitwise
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402

N = int(os.environ.get("REPEAT_N", "200"))
M = int(os.environ.get("REPEAT_M", "40"))


def main():
    dev = torch.device("cuda", 0)
    B, V, D, H, W = 4, 3, 192, 512, 640
    net = bench.build_model(D, H, W, dev)
    inputs = bench.make_inputs(B, V, H, W, 0, dev)
    probs = []
    hook = net.cost_volume_reg.register_forward_hook(lambda m, i, o: probs.append(o))
    bad = 0
    with torch.no_grad():
        ini0, ref0 = net(*inputs, B, V)
        p0 = probs.pop().clone()
        for r in range(N):
            ini, ref = net(*inputs, B, V)
            p = probs.pop()
            ok = torch.equal(p, p0) and torch.equal(ini, ini0) and torch.equal(ref, ref0)
            if not ok:
                bad += 1
                d = (p != p0)
                idx = d.nonzero()[:8].tolist()
                print("eval run %d differs: %d P voxels (first %s), depth %d px" % (
                    r, int(d.sum()), idx, int((ini != ini0).sum())), flush=True)
    hook.remove()
    print("eval step: %d of %d runs differ" % (bad, N), flush=True)
    del net
    from mvs_amd import ops
    from cameras import camera_batch, depth_range
    h, w, C = H // 4, W // 4, 32
    K, R, T = camera_batch(B, V, h, w)
    d_min, d_int = depth_range(B)
    g = torch.Generator(device="cpu").manual_seed(3)
    feat = torch.randn(B * V, C, h, w, generator=g).to(dev)
    gcv = torch.randn(B, C, D, h, w, generator=g).to(dev)
    _, ws = ops.cost_volume(feat, K, R, T, d_min, d_int, B, V, 0, D, 25.0)
    g0 = ops.cost_volume_backward(feat, ws, gcv, B, V, D, True)
    bad = 0
    for r in range(M):
        gr = ops.cost_volume_backward(feat, ws, gcv, B, V, D, True)
        if not torch.equal(gr, g0):
            bad += 1
            print("backward run %d differs: %d elements" % (r, int((gr != g0).sum())), flush=True)
    print("deterministic backward: %d of %d runs differ" % (bad, M), flush=True)


if __name__ == "__main__":
    main()
