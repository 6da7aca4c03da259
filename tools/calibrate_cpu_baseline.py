"""Calibration gate of the CPU baseline (BASELINE.md "CPU-baseline plan"), run in the SURVEY
container only (it imports the reference from /root/reference, which does not exist on the GPU box).

Times, on the same host and thread count, at config 1 (B=1, V=3, 640x512 images, D=48) with the
weights of tests/golden/weights.py and the inputs of tests/golden/make_golden.py::case_cfg1_e2e:
  * the REFERENCE's own MVSNet.forward (scripts/model.py, kornia 0.6.3 stand-in = the oracle's
    restatement, config patched before import) -- one warm-up, median of 3;
  * the oracle's forward (oracle/mvs_oracle.py::mvsnet_forward, concat_growth=True: the build's
    CPU restatement that bench.py times on the GPU box) -- one warm-up, median of 3;
  * both sides' warp (homography_warping) and variance alone.
The restatement passes the gate when its full forward is within +-15 % of the reference's.
Writes profiles/cpu_calibration_r02.json.

Run:  PYTHONDONTWRITEBYTECODE=1 python tools/calibrate_cpu_baseline.py [threads]
"""
import json
import os
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("deep-multiview-depth-estimation_amd", "oracle", os.path.join("tests", "golden")):
    sys.path.insert(0, os.path.join(REPO, sub))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def median_time(fn, reps=3):
    fn()   # warm-up
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return statistics.median(ts), ts


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else (os.cpu_count() or 1)
    torch.set_num_threads(threads)
    import make_golden
    import mvs_oracle
    from cameras import camera_batch, depth_range
    from weights import deterministic_state_dict
    from mvs_amd.config import MVSConfig
    from mvs_amd.model import MVSNet
    B, V, D = 1, 3, 48
    _, ref_h, ref_cv, _ = make_golden._import_reference(D, 128, 160)
    import model as ref_model
    ref_net = ref_model.MVSNet()
    ref_net.load_state_dict(deterministic_state_dict(ref_net.state_dict()))
    ref_net.eval()
    net = MVSNet(MVSConfig(d_num=D), device=torch.device("cpu"))
    net.load_state_dict(deterministic_state_dict(net.state_dict()))
    net.eval()
    K, R, T = camera_batch(B, V, 128, 160)
    d_min, d_int = depth_range(B)
    img = torch.from_numpy(np.random.default_rng(11).standard_normal((B * V, 3, 512, 640), dtype=np.float32))
    out = {"config": "cfg1: B=1, V=3, 640x512, D=48, BN eval, no_grad", "threads": threads,
           "torch": torch.__version__, "cpu": _cpu_model()}
    with torch.no_grad():
        feats = net.feature_encoder(img)
        out["reference_forward_s"], out["reference_forward_runs"] = median_time(
            lambda: ref_net(img, K, R, T, d_min, d_int, B, V))
        out["oracle_forward_s"], out["oracle_forward_runs"] = median_time(
            lambda: mvs_oracle.mvsnet_forward(net, img, K, R, T, d_min, d_int, B, V, D, (128, 160),
                                              concat_growth=True))
        out["reference_warp_variance_s"], _ = median_time(
            lambda: ref_cv.assemble_cost_volume(
                ref_h.homography_warping(K, R, T, d_min, d_int, feats, B, V, d_num=D)[0], V))
        out["oracle_warp_variance_s"], _ = median_time(
            lambda: mvs_oracle.assemble_cost_volume(
                mvs_oracle.homography_warping(K, R, T, d_min, d_int, feats, B, V, D, concat_growth=True)[0], V))
    out["ratio_forward"] = out["oracle_forward_s"] / out["reference_forward_s"]
    out["ratio_warp_variance"] = out["oracle_warp_variance_s"] / out["reference_warp_variance_s"]
    out["gate_pass"] = abs(out["ratio_forward"] - 1.0) <= 0.15
    path = os.path.join(REPO, "profiles", "cpu_calibration_r02.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


def _cpu_model():
    try:
        txt = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        return {k.strip(): v.strip() for k, v in (l.split(":", 1) for l in txt.splitlines() if ":" in l)
                if k.strip() in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "CPU(s)")}
    except (OSError, subprocess.SubprocessError):
        return {}


if __name__ == "__main__":
    main()
