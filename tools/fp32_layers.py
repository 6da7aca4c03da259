"""Per-layer GPU time of the fp32 live-region regulariser (CostVolumeReg._forward_live_hip in the default
fp32 arithmetic) at cfg 2 (B=4, fp32 channel-quad cost volume 32 x 192 x 128 x 160): each layer ALONE
(back-to-back launches, HIP events), the LDS-staged stride-1 kernels against the per-lane ones (and their
bit-equality), then the whole fp32 eval step with conv_0_0 on its side stream (as shipped) and serialised.

Usage: python tools/fp32_layers.py [--reps N] [--only NAME[,NAME]]   (env MVS_T2_RB=4 etc. for A/B builds)
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402
from mvs_amd import model as M  # noqa: E402
from mvs_amd.ops import (CONV_S1, CONV_S2, CONV_T2, conv3d_k3, conv3d_region, conv_head_fp32,  # noqa: E402
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
    print("%-34s %8.3f ms" % (name, e0.elapsed_time(e1) / n), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B, V, D, H, W = 4, 3, 192, 512, 640
    net = bench.build_model(D, H, W, dev)
    img, K, R, T, d_min, d_int = bench.make_inputs(B, V, H, W, 0, dev)
    reg = net.cost_volume_reg
    from mvs_amd import warp_and_assemble_cost_volume
    with torch.no_grad():
        feats = net.feature_encoder(img)
        cv = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, feats, B, V, d_num=D, channel_quads=True)[0].data
        n = tuple(cv.shape[2:5])
        full = tuple((0, d - 1) for d in n)
        Bq = M._tconv_input_region(full, n, reg.pad)
        C2 = M._tconv_input_region(Bq, n, reg.pad)
        C3 = M._tconv_input_region(C2, n, reg.pad)
        org = lambda r: [lo for lo, _ in r]
        size = lambda r: [hi - lo + 1 for lo, hi in r]
        dims, pad = list(n), list(reg.pad)
        bn = M._bn_eval
        layers = {"conv_0_0": lambda: conv3d_k3(cv, reg.conv_0_0.weight, *bn(reg.BN_0), in_c4=True, wino_z=True)}
        y0 = layers["conv_0_0"]()
        h1 = M._grow(Bq, n, 1)
        layers["conv_head"] = lambda: conv_head_fp32(cv, reg.conv_0_0.weight, *bn(reg.BN_0), reg.conv_1_0.weight,
                                                     *bn(reg.BN_1), pad, org(h1), size(h1))
        lv = []
        for k, (ca, cb, bnm, r) in enumerate(((reg.conv_1_0, reg.conv_1_1, reg.BN_1, Bq),
                                              (reg.conv_2_0, reg.conv_2_1, reg.BN_2, C2),
                                              (reg.conv_3_0, reg.conv_3_1, reg.BN_3, C3))):
            halo = M._grow(r, n, 1)
            fa = (lambda ca=ca, bnm=bnm, halo=halo: conv3d_region(
                cv, None, region_weight(ca), CONV_S2, dims, org(halo), size(halo), None, None, pad, *bn(bnm), in_c4=True))
            ya = fa()
            layers["conv_%d_0" % (k + 1)] = fa
            for lane_kind in (False, True):
                fb = (lambda cb=cb, bnm=bnm, halo=halo, r=r, ya=ya, pl=lane_kind: conv3d_region(
                    ya, None, region_weight(cb), CONV_S1, dims, org(r), size(r), org(halo), size(halo), None, *bn(bnm),
                    out_ncdhw=r is Bq, per_lane=pl))
                layers["conv_%d_1%s" % (k + 1, "_per_lane" if lane_kind else "")] = fb
            y_lds = layers["conv_%d_1" % (k + 1)]()
            y_pl = layers["conv_%d_1_per_lane" % (k + 1)]()
            print("conv_%d_1 LDS vs per-lane: bit-equal %s (max|d| %.3g)" % (
                k + 1, torch.equal(y_lds, y_pl), (y_lds - y_pl).abs().max().item()), flush=True)
            lv.append(y_lds)
        y1, y2, y3 = lv
        layers["deconv_3_0"] = lambda: conv3d_region(y3, None, region_weight(reg.deconv_3_0), CONV_T2, dims, org(C2),
                                                     size(C2), org(C3), size(C3), pad, *bn(reg.BN_2))
        y3b = layers["deconv_3_0"]()
        layers["deconv_2_0"] = lambda: conv3d_region(y3b, y2, region_weight(reg.deconv_2_0), CONV_T2, dims, org(Bq),
                                                     size(Bq), org(C2), size(C2), pad, *bn(reg.BN_1), out_ncdhw=True)
        y2b = layers["deconv_2_0"]()
        print("deconv sha: %.9g %.9g" % (y3b.double().sum().item(), y2b.double().sum().item()), flush=True)
        layers["deconv_1_0"] = lambda: deconv3d_k3s2(y2b, org(Bq), reg.deconv_1_0.weight, dims, pad, *bn(reg.BN_0), y0,
                                                     x2=y1)
        z = layers["deconv_1_0"]()
        layers["conv_out"] = lambda: conv3d_k3(z, reg.conv_out.weight)
        o = layers["conv_out"]()
        layers["softmax"] = lambda: softmax_depth(o)
        layers["encoder"] = lambda: net.feature_encoder(img)
        layers["cost_volume"] = lambda: warp_and_assemble_cost_volume(K, R, T, d_min, d_int, feats, B, V, d_num=D,
                                                                      channel_quads=True)
        step = lambda: net(img, K, R, T, d_min, d_int, B, V)
        layers["step"] = step
        yh0, yh1 = layers["conv_head"]()
        print("conv_head: y0 bit-equal %s, y1 max|d| vs conv_1_0 %.3g" % (
            torch.equal(yh0, y0), (yh1 - layers["conv_1_0"]()).abs().max().item()), flush=True)
        names = a.only.split(",") if a.only else list(layers)
        for name in names:
            timed(name, layers[name], a.reps)
        if a.only:
            return
        saved = M._side_stream
        M._side_stream = lambda device, which=0, priority=0: torch.cuda.current_stream(device)
        try:
            timed("eval step (serialised)", step, a.reps)
        finally:
            M._side_stream = saved


if __name__ == "__main__":
    main()
