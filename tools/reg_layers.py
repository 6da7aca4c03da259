"""Per-layer GPU time of the eval-mode live-region regulariser at cfg 2 (B=4, 32 x 192 x 128 x 160).

Usage: python tools/reg_layers.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "deep-multiview-depth-estimation_amd"))
import bench  # noqa: E402,F401  (MIOPEN_USER_DB_PATH -> tools/miopen_db)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402,F401
from mvs_amd import model as M  # noqa: E402
from mvs_amd.config import pad_outpad  # noqa: E402


def timed(name, fn, n=3):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        out = fn()
    e1.record()
    torch.cuda.synchronize()
    print("%-34s %8.3f ms" % (name, e0.elapsed_time(e1) / n), flush=True)
    return out


def main():
    dev = torch.device("cuda", 0)
    B, D, h, w = 4, 192, 128, 160
    pad, outpad = pad_outpad(D, h, w)
    reg = M.CostVolumeReg(pad=pad, outpad=outpad).to(dev).eval()
    cv = torch.randn(B, 32, D, h, w, device=dev)
    n = (D, h, w)
    full = tuple((0, d - 1) for d in n)
    Bq = M._tconv_input_region(full, n, pad)
    C2 = M._tconv_input_region(Bq, n, pad)
    C3 = M._tconv_input_region(C2, n, pad)
    print("regions", Bq, C2, C3, flush=True)
    with torch.no_grad():
        y0 = timed("conv_0_0 full (MIOpen)", lambda: reg.conv_0_0(cv))
        from mvs_amd.ops import conv3d_k3
        y0h = timed("conv_0_0 full (HIP conv3d_k3)", lambda: conv3d_k3(cv, reg.conv_0_0.weight))
        print("  max |HIP - MIOpen| %.3g (max %.3g)" % ((y0h - y0).abs().max().item(), y0.abs().max().item()))
        timed("bn+relu y0", lambda: reg.ReLU(reg.BN_0(y0)))
        ys = []
        for k, (ca, cb, bn, r) in enumerate(((reg.conv_1_0, reg.conv_1_1, reg.BN_1, Bq),
                                             (reg.conv_2_0, reg.conv_2_1, reg.BN_2, C2),
                                             (reg.conv_3_0, reg.conv_3_1, reg.BN_3, C3))):
            halo = M._grow(r, n, 1)
            y = timed("conv_%d_0 region" % (k + 1), lambda: M._conv_s2_region(cv, ca.weight, halo, pad))
            y = reg.ReLU(bn(y))
            ys.append(timed("conv_%d_1 region" % (k + 1), lambda: M._conv_s1_region(y, halo, cb.weight, r, n)))
        y1, y2, y3 = ys
        y3 = timed("deconv_3_0", lambda: M._tconv_region(y3, C3, reg.deconv_3_0.weight, C2, pad))
        y2 = timed("deconv_2_0", lambda: M._tconv_region(y3 + y2, C2, reg.deconv_2_0.weight, Bq, pad))
        y1 = timed("deconv_1_0 (full output)", lambda: M._tconv_region(y2 + y1, Bq, reg.deconv_1_0.weight, full, pad))
        z = timed("add y1+y0", lambda: y1 + y0)
        o = timed("conv_out full (MIOpen)", lambda: reg.conv_out(z))
        timed("conv_out full (HIP conv3d_k3)", lambda: conv3d_k3(z, reg.conv_out.weight))
        timed("softmax", lambda: reg.Norm(o))
        timed("whole forward_live", lambda: reg(cv))


if __name__ == "__main__":
    main()
