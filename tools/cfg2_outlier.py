"""Why is the GPU's worst unflipped cfg-2 pixel (against the float64 law) far off?  

Reads the worst-pixel records of test_cfg2_depth_flips_within_reference_self_noise
(<parity dir>/cfg2_vs_float64_law.json: per sample the pixel, the GPU's 8 most probable planes and
their P, the kept planes of the GPU / f64 / fp32 reference, the three depths), recomputes that
sample on the CPU -- the fp32 oracle (the reference's numerics), the same with the fp64-composed
sampling matrices (hom64), and the float64 law -- and prints, at the pixel:

  * P of the kept planes in each model, the depth sum(d_k P_k) / sum(P_k) over them;
  * the depth's sensitivity to the kept planes' relative P error eps: sum|d_k - d| P_k / sum P_k
    (a 1e-5 relative P change moves the depth by 1e-5 x this);
  * the logit gap of the softmax around the kept planes (P ratios), i.e. how close the pixel is to a
    near-tie that the random-weight network amplifies.

Usage: python tools/cfg2_outlier.py gpurun_out/<tag>/parity [sample ...]   (~6 min per sample, 8 cores)
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("deep-multiview-depth-estimation_amd", "oracle", os.path.join("tests", "golden")):
    sys.path.insert(0, os.path.join(REPO, sub))


def main():
    rec = json.load(open(os.path.join(sys.argv[1], "cfg2_vs_float64_law.json")))
    samples = [int(s) for s in sys.argv[2:]] or [int(np.argmax(rec["gpu_max_rel_unflipped"]))]
    import copy
    import mvs_oracle
    from make_cfg2_selfnoise import GEOM, cfg2_inputs
    B, V, D, H, W = GEOM
    h, w = H // 4, W // 4
    net, img, K, R, T, d_min, d_int = cfg2_inputs()
    net64 = copy.deepcopy(net).double().eval()
    torch.set_num_threads(os.cpu_count() or 8)
    for b in samples:
        px = rec["gpu_worst_unflipped_pixel"][b]
        y, x = px["y"], px["x"]
        sl = slice(b * V, (b + 1) * V)
        args = (img[sl], K[sl], R[sl], T[sl], d_min[b:b + 1], d_int[b:b + 1], 1, V, D, (h, w))
        with torch.no_grad():
            i32, _, p32 = mvs_oracle.mvsnet_forward(net, *args)
            ih, _, ph = mvs_oracle.mvsnet_forward(net, *args, hom64=True)
            i64, _, p64 = mvs_oracle.mvsnet_forward64(net64, *args)
        dk = mvs_oracle.depth_planes(d_min[b:b + 1].double(), d_int[b:b + 1].double(), D)[0, :, 0, 0].numpy()
        print("sample %d pixel (y=%d, x=%d): GPU depth %.4f, f64 %.4f, fp32 ref %.4f (GPU rel %.3g)" % (
            b, y, x, px["depth_gpu"], px["depth_f64"], px["depth_fp32_ref"],
            abs(px["depth_gpu"] - px["depth_f64"]) / abs(px["depth_f64"])))
        for name, P, dep in (("fp32 ref", p32, i32), ("fp32 ref hom64", ph, ih), ("float64 law", p64, i64)):
            pv = P[0, 0, :, y, x].double().numpy()
            top = np.argsort(-pv, kind="stable")[:8]
            kept = np.sort(top[:5])
            d = float((dk[kept] * pv[kept]).sum() / pv[kept].sum())
            sens = float((np.abs(dk[kept] - d) * pv[kept]).sum() / pv[kept].sum())
            print("  %-15s depth %.4f (model %.4f) kept %s P %s" % (name, d, float(dep[0, 0, y, x]), kept.tolist(),
                                                                 np.array2string(pv[kept], precision=4)))
            print("  %-15s top8 %s  P %s  sensitivity sum|d_k-d|P_k/sumP = %.1f mm (x eps)" % (
                "", top.tolist(), np.array2string(pv[top], precision=3), sens))
        print("  GPU            top8 %s  P %s" % (px["gpu_top8_planes"], np.array2string(np.array(px["gpu_top8_p"]),
                                                                                       precision=3)))


if __name__ == "__main__":
    main()
