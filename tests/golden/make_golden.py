"""Generate golden vectors by running the REFERENCE's own Python on the CPU (survey container only).

Imports ``/root/reference/scripts/{config,homography,costvolume,depthmap,model}.py`` unmodified.
``kornia`` (0.6.3, pinned at ``requirements.txt:1``) is absent here, so a stand-in module
``kornia.geometry.transform`` exposing ``oracle/kornia_warp.warp_perspective`` is registered in
``sys.modules`` before the import (SURVEY.md §8 c).  ``config`` is patched (D_NUM, FEAT_H/W,
PAD/OUTPAD, DEVICE=cpu) before ``homography``/``model`` are imported, because they bind those
constants at import time (``homography.py:3,14``, ``model.py:10``).  Each case runs in a fresh
subprocess so every case gets its own config.

Outputs (small .npz, committed):
  tiny_v3.npz / tiny_v5.npz  full tensors: B=2 with distinct d_min/d_int (pins the i mod B plane
                             tiling), C=8, 12x16, D=6, real DTU cameras rescaled
  softargmin.npz             depthmap.extract_depth_map known answers (SURVEY a7 example, ties,
                             random, D == N_DEPTH_EST)
  cfg1_cv.npz                config-1 cost volume (B=1,V=3,C=32,128x160,D=48): 4096 seeded voxel
                             samples + sum, sum of squares, max
  state_dict_keys.json       the reference MVSNet state_dict keys/shapes (D_NUM=20) and parameter count
  cfg1_e2e.npz               MVSNet.forward at config 1 (640x512 images, D=48) with the weights of
                             tests/golden/weights.py: initial/refined depth, BN eval mode and the
                             test.py:61 train-mode-under-no_grad mode

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
import os
import subprocess
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/scripts"


def _install_kornia_standin():
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import kornia_warp
    k = types.ModuleType("kornia")
    kg = types.ModuleType("kornia.geometry")
    kgt = types.ModuleType("kornia.geometry.transform")
    kgt.warp_perspective = kornia_warp.warp_perspective
    k.geometry = kg
    kg.transform = kgt
    sys.modules.update({"kornia": k, "kornia.geometry": kg, "kornia.geometry.transform": kgt})


def _import_reference(d_num, feat_h=128, feat_w=160, in_h=512, in_w=640):
    import torch
    _install_kornia_standin()
    sys.path.insert(0, REF)
    import config
    config.D_NUM = d_num
    config.IN_H, config.IN_W = in_h, in_w
    config.FEAT_H, config.FEAT_W = feat_h, feat_w
    dims = np.array([d_num, feat_h, feat_w])
    config.PAD = tuple(np.int64(np.floor(dims / 2) + 1))
    config.OUTPAD = tuple((dims + 1) % 2)
    config.DEVICE = torch.device("cpu")
    import homography
    import costvolume
    import depthmap
    return config, homography, costvolume, depthmap


def case_tiny(n_views):
    import torch
    sys.path.insert(0, HERE)
    from cameras import camera_batch, depth_range, features
    B, C, h, w, D = 2, 8, 12, 16, 6
    _, homography, costvolume, _ = _import_reference(D, h, w)
    K, R, T = camera_batch(B, n_views, h, w)
    d_min, d_int = depth_range(B, distinct=True)
    d_int = d_int * 25.0       # spread the 6 planes over ~[425, 1500] mm at this tiny size
    feat = features(B * n_views, C, h, w, seed=10 + n_views)
    with torch.no_grad():
        warped, d_batch_0, ref_idx_0 = homography.homography_warping(
            K, R, T, d_min, d_int, feat, B, n_views, d_num=D)
        cv = costvolume.assemble_cost_volume(warped, n_views)
    np.savez_compressed(os.path.join(HERE, "tiny_v%d.npz" % n_views),
                        feat=feat.numpy(), K=K.numpy(), R=R.numpy(), T=T.numpy(),
                        d_min=d_min.numpy(), d_int=d_int.numpy(), d_num=D, batch_size=B,
                        n_views=n_views, warped=warped.numpy(), d_batch_0=d_batch_0.numpy(),
                        ref_idx_0=ref_idx_0.numpy(), cv=cv.numpy())


def case_softargmin():
    import torch
    config, _, _, depthmap = _import_reference(8)
    out = {}
    # SURVEY §8 a7 worked example (permutation-indexed mask, not a true top-5)
    p = torch.tensor([.01, .02, .3, .05, .4, .1, .07, .05]).reshape(1, 1, 8, 1, 1)
    d = (425.0 + 25.0 * torch.arange(8.0)).reshape(1, 8, 1, 1)
    out["ex_p"], out["ex_d"] = p.numpy(), d.numpy()
    out["ex_depth"] = depthmap.extract_depth_map(p, d).numpy()
    # random, D = 10
    g = torch.Generator().manual_seed(7)
    p = torch.softmax(torch.randn(2, 1, 10, 4, 5, generator=g), dim=2)
    d = (300.0 + 40.0 * torch.arange(10.0)).reshape(1, 10, 1, 1).repeat(2, 1, 1, 1)
    d[1] += 100.0
    out["rnd_p"], out["rnd_d"] = p.numpy(), d.numpy()
    out["rnd_depth"] = depthmap.extract_depth_map(p, d).numpy()
    # exact ties: a uniform column and a two-level column
    p = torch.full((1, 1, 12, 1, 2), 1.0 / 12)
    p[0, 0, ::2, 0, 1] = 0.1
    p[0, 0, 1::2, 0, 1] = 1.0 / 15
    d = (500.0 + 10.0 * torch.arange(12.0)).reshape(1, 12, 1, 1)
    out["tie_p"], out["tie_d"] = p.numpy(), d.numpy()
    out["tie_depth"] = depthmap.extract_depth_map(p, d).numpy()
    # D == N_DEPTH_EST: every plane kept -> plain soft-argmin
    p = torch.softmax(torch.randn(1, 1, 5, 3, 3, generator=g), dim=2)
    d = (425.0 + 25.0 * torch.arange(5.0)).reshape(1, 5, 1, 1)
    out["d5_p"], out["d5_d"] = p.numpy(), d.numpy()
    out["d5_depth"] = depthmap.extract_depth_map(p, d).numpy()
    out["n_depth_est"] = int(config.N_DEPTH_EST)
    np.savez_compressed(os.path.join(HERE, "softargmin.npz"), **out)


def case_cfg1_cv():
    import torch
    sys.path.insert(0, HERE)
    from cameras import camera_batch, depth_range, features
    B, V, C, h, w, D = 1, 3, 32, 128, 160, 48
    _, homography, costvolume, _ = _import_reference(D, h, w)
    K, R, T = camera_batch(B, V, h, w)
    d_min, d_int = depth_range(B)
    feat = features(B * V, C, h, w, seed=1)
    with torch.no_grad():
        warped, _, _ = homography.homography_warping(K, R, T, d_min, d_int, feat, B, V, d_num=D)
        cv = costvolume.assemble_cost_volume(warped, V)
    cv64 = cv.double()
    rng = np.random.default_rng(4096)
    idx = rng.integers(0, cv.numel(), size=4096)
    np.savez_compressed(os.path.join(HERE, "cfg1_cv.npz"), K=K.numpy(), R=R.numpy(), T=T.numpy(),
                        d_min=d_min.numpy(), d_int=d_int.numpy(), feat_seed=1,
                        shape=np.array(cv.shape), sample_idx=idx,
                        sample_val=cv.reshape(-1)[torch.from_numpy(idx)].numpy(),
                        total=float(cv64.sum()), total_sq=float((cv64 * cv64).sum()),
                        vmax=float(cv.max()))


def case_cfg1_e2e():
    import torch
    sys.path.insert(0, HERE)
    from cameras import camera_batch, depth_range
    from weights import deterministic_state_dict
    B, V, D = 1, 3, 48
    _import_reference(D, 128, 160)
    import model as ref_model
    torch.manual_seed(0)
    net = ref_model.MVSNet()
    net.load_state_dict(deterministic_state_dict(net.state_dict()))
    K, R, T = camera_batch(B, V, 128, 160)
    d_min, d_int = depth_range(B)
    rng = np.random.default_rng(11)
    img = torch.from_numpy(rng.standard_normal((B * V, 3, 512, 640), dtype=np.float32))
    out = dict(K=K.numpy(), R=R.numpy(), T=T.numpy(), d_min=d_min.numpy(), d_int=d_int.numpy(),
               img_seed=11, weight_seed=1234, d_num=D)
    with torch.no_grad():
        net.eval()
        ini, ref = net(img, K, R, T, d_min, d_int, B, V)
        out["eval_initial"], out["eval_refined"] = ini.numpy(), ref.numpy()
        net.train()     # test.py:61 -- BatchNorm in train mode under no_grad
        ini, ref = net(img, K, R, T, d_min, d_int, B, V)
        out["train_initial"], out["train_refined"] = ini.numpy(), ref.numpy()
    np.savez_compressed(os.path.join(HERE, "cfg1_e2e.npz"), **out)


def case_state_dict_keys():
    import json
    _import_reference(20, 128, 160)
    import model as ref_model
    net = ref_model.MVSNet()
    keys = [[k, list(v.shape)] for k, v in net.state_dict().items()]
    n_params = sum(p.numel() for p in net.parameters)
    with open(os.path.join(HERE, "state_dict_keys.json"), "w") as f:
        json.dump({"keys": keys, "n_params": n_params, "d_num": 20}, f, indent=0)


CASES = {"keys": case_state_dict_keys, "tiny_v3": lambda: case_tiny(3), "tiny_v5": lambda: case_tiny(5),
         "softargmin": case_softargmin, "cfg1_cv": case_cfg1_cv, "cfg1_e2e": case_cfg1_e2e}


if __name__ == "__main__":
    if len(sys.argv) > 1:
        CASES[sys.argv[1]]()
        print("ok", sys.argv[1])
    else:
        env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
        for name in CASES:
            subprocess.check_call([sys.executable, os.path.abspath(__file__), name], env=env,
                                  cwd="/tmp")
