"""Per-layer GPU time of the HIP live-region regulariser (CostVolumeReg._forward_live_hip) at cfg 2
(B=4, channel-quad cost volume 32 x 192 x 128 x 160), each layer ALONE (back-to-back launches, HIP
events), then the whole eval step with conv_0_0 on its side stream (as shipped) and serialised on the
main stream -- how much the concurrency buys and what each layer costs without a neighbour.

Usage: python tools/hip_reg_layers.py [--only NAME] [--reps N]
  --only conv_1_0   run just that layer N times (for rocprofv3 --pmc passes on one kernel)
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402
from mvs_amd import model as M  # noqa: E402
from mvs_amd.ops import conv_s2_split, split_head  # noqa: E402
from mvs_amd.ops import (CONV_S1, CONV_S2, CONV_T2, conv3d_k3, conv3d_k3_split, conv3d_region,  # noqa: E402
                         deconv3d_k3s2, region_weight, softmax_depth)


def timed(name, fn, n):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        out = fn()
    e1.record()
    torch.cuda.synchronize()
    print("%-28s %8.3f ms" % (name, e0.elapsed_time(e1) / n), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B, V, D, H, W = 4, 3, 192, 512, 640
    net = bench.build_model(D, H, W, dev)
    img, K, R, T, d_min, d_int = bench.make_inputs(B, V, H, W, 0, dev)
    reg = net.cost_volume_reg
    from mvs_amd import warp_and_assemble_cost_volume
    with torch.no_grad():
        feats = net.feature_encoder(img)
        cv, _, _ = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, feats, B, V, d_num=D, channel_quads=True)
        cvs, _, _ = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, feats, B, V, d_num=D, channel_quads=True,
                                                  split=True)
        cv, cvs, bound = cv.data, cvs.data, cvs.absmax   # BoundCostVolume: (volume, bound words)
        n = tuple(cv.shape[2:5])
        full = tuple((0, d - 1) for d in n)
        Bq = M._tconv_input_region(full, n, reg.pad)
        C2 = M._tconv_input_region(Bq, n, reg.pad)
        C3 = M._tconv_input_region(C2, n, reg.pad)
        org = lambda r: [lo for lo, _ in r]
        size = lambda r: [hi - lo + 1 for lo, hi in r]
        dims, pad = list(n), list(reg.pad)
        bn = M._bn_eval
        layers = {}
        layers["conv_0_0"] = lambda: conv3d_k3(cv, reg.conv_0_0.weight, *bn(reg.BN_0), in_c4=True, wino_z=True)
        layers["conv_0_0_split"] = lambda: conv3d_k3_split(cvs, bound, reg.conv_0_0.weight, *bn(reg.BN_0))
        y0 = layers["conv_0_0"]()
        y0s = layers["conv_0_0_split"]()
        print("conv_0_0 split vs exact fp32: max|d| %.3g (max|y| %.3g)"
              % ((y0s - y0).abs().max().item(), y0.abs().max().item()), flush=True)
        lv = []
        for k, (ca, cb, bnm, r) in enumerate(((reg.conv_1_0, reg.conv_1_1, reg.BN_1, Bq),
                                              (reg.conv_2_0, reg.conv_2_1, reg.BN_2, C2),
                                              (reg.conv_3_0, reg.conv_3_1, reg.BN_3, C3))):
            halo = M._grow(r, n, 1)
            fa = (lambda ca=ca, bnm=bnm, halo=halo: conv3d_region(
                cv, None, region_weight(ca), CONV_S2, dims, org(halo), size(halo), None, None, pad, *bn(bnm), in_c4=True))
            ya = fa()
            fb = (lambda cb=cb, bnm=bnm, halo=halo, r=r, ya=ya: conv3d_region(
                ya, None, region_weight(cb), CONV_S1, dims, org(r), size(r), org(halo), size(halo), None, *bn(bnm),
                out_ncdhw=r is Bq))
            layers["conv_%d_0" % (k + 1)] = fa
            if k == 0:
                layers["conv_1_0_split"] = (lambda ca=ca, bnm=bnm, halo=halo: conv_s2_split(
                    cvs, bound, ca.weight, dims, org(halo), size(halo), pad, *bn(bnm)))
                ys = layers["conv_1_0_split"]()
                print("conv_1_0 split vs exact fp32: max|d| %.3g (max|y| %.3g)"
                      % ((ys - ya).abs().max().item(), ya.abs().max().item()), flush=True)
            layers["conv_%d_1" % (k + 1)] = fb
            lv.append(fb())
        y1, y2, y3 = lv
        layers["deconv_3_0"] = lambda: conv3d_region(y3, None, region_weight(reg.deconv_3_0), CONV_T2, dims, org(C2),
                                                     size(C2), org(C3), size(C3), pad, *bn(reg.BN_2))
        y3b = layers["deconv_3_0"]()
        layers["deconv_2_0"] = lambda: conv3d_region(y3b, y2, region_weight(reg.deconv_2_0), CONV_T2, dims, org(Bq),
                                                     size(Bq), org(C2), size(C2), pad, *bn(reg.BN_1), out_ncdhw=True)
        y2b = layers["deconv_2_0"]()
        layers["deconv_1_0"] = lambda: deconv3d_k3s2(y2b, org(Bq), reg.deconv_1_0.weight, dims, pad, *bn(reg.BN_0), y0,
                                                     x2=y1)
        z = layers["deconv_1_0"]()
        layers["conv_out"] = lambda: conv3d_k3(z, reg.conv_out.weight)
        o = layers["conv_out"]()
        layers["softmax"] = lambda: softmax_depth(o)
        # the fused head (csrc/cv_head.hip): variance + conv_0_0 + conv_1_0 on chip, against the split
        # producer + the two split consumers it replaces
        dcv, _, _ = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, feats, B, V, d_num=D, deferred=True)
        h1, h2 = M._grow(Bq, n, 1), M._grow(C2, n, 1)
        lo = [max(2 * a0 - p, 0) for (a0, _), p in zip(h2, pad)]
        hi = [min(2 * b1 - p + 2, d - 1) + 1 for (_, b1), p, d in zip(h2, pad, n)]
        layers["cv_split"] = lambda: warp_and_assemble_cost_volume(K, R, T, d_min, d_int, feats, B, V, d_num=D,
                                                                   channel_quads=True, split=True)
        layers["cv_head"] = lambda: dcv.head(reg.conv_0_0.weight, bn(reg.BN_0), reg.conv_1_0.weight, bn(reg.BN_1),
                                             pad, org(h1), size(h1), lo, hi)
        y0h, y1h, box = layers["cv_head"]()
        y1s = conv_s2_split(cvs, bound, reg.conv_1_0.weight, dims, org(h1), size(h1), pad, *bn(reg.BN_1))
        sl = (slice(None), slice(None)) + tuple(slice(a0, b1) for a0, b1 in zip(lo, hi))
        print("cv_head vs split path: y0 equal %s (max|d| %.3g), y1 equal %s (max|d| %.3g), box equal %s" % (
            torch.equal(y0h, y0s), (y0h - y0s).abs().max().item(), torch.equal(y1h, y1s),
            (y1h - y1s).abs().max().item(), torch.equal(box.data, cvs[sl])), flush=True)
        layers["split_head"] = lambda: split_head(cvs, bound, reg.conv_0_0.weight, *bn(reg.BN_0), reg.conv_1_0.weight,
                                                  *bn(reg.BN_1), pad, org(h1), size(h1))
        y0p, y1p = layers["split_head"]()
        print("split_head vs split path: y0 equal %s, y1 equal %s" % (torch.equal(y0p, y0s), torch.equal(y1p, y1s)),
              flush=True)
        if a.only:   # one layer or a comma-separated list ("step": the whole eval step)
            for name in a.only.split(","):
                timed(name, (lambda: net(img, K, R, T, d_min, d_int, B, V)) if name == "step" else layers[name],
                      a.reps)
            return
        for name, fn in layers.items():
            timed(name, fn, a.reps)
        step = lambda: net(img, K, R, T, d_min, d_int, B, V)
        timed("eval step (split volume + split head)", step, a.reps)
        os.environ["MVS_SPLIT_HEAD"] = "0"
        timed("eval step (split volume, separate conv_0_0 / conv_1_0)", step, a.reps)
        os.environ.pop("MVS_SPLIT_HEAD")
        os.environ["MVS_CV_HEAD"] = "1"
        timed("eval step (opt-in fused gather head)", step, a.reps)
        os.environ.pop("MVS_CV_HEAD")
        reg.split_f16 = False
        timed("eval step (exact fp32 conv_0_0)", step, a.reps)
        reg.split_f16 = True
        saved = M._side_stream
        M._side_stream = lambda device, which=0, priority=0: torch.cuda.current_stream(device)
        try:
            timed("eval step (serialised)", step, a.reps)
        finally:
            M._side_stream = saved


if __name__ == "__main__":
    main()
