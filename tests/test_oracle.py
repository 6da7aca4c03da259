"""CPU: pin the oracle (oracle/) against the reference-generated golden vectors and analytic
known answers.  The kornia 0.6.3 internals are parity-unpinned against real kornia (absent); the
known-answer tests below pin the sampling law they implement."""
import numpy as np
import pytest
import torch

import kornia_warp
import mvs_oracle
from conftest import load_golden


def _t(z, k):
    return torch.from_numpy(np.asarray(z[k]))


@pytest.mark.parametrize("nv", [3, 5])
def test_oracle_matches_reference_golden_tiny(nv):
    z = load_golden("tiny_v%d.npz" % nv)
    B, D = int(z["batch_size"]), int(z["d_num"])
    warped, d_batch_0, ref_idx_0 = mvs_oracle.homography_warping(
        _t(z, "K"), _t(z, "R"), _t(z, "T"), _t(z, "d_min"), _t(z, "d_int"), _t(z, "feat"), B, nv, D)
    cv = mvs_oracle.assemble_cost_volume(warped, nv)
    # same op sequence as the reference on the same library: bit-exact
    assert np.array_equal(warped.numpy(), z["warped"])
    assert np.array_equal(cv.numpy(), z["cv"])
    assert np.array_equal(d_batch_0.numpy(), z["d_batch_0"])
    assert np.array_equal(ref_idx_0.numpy(), z["ref_idx_0"])


def test_golden_pins_plane_tiling_quirk():
    """homography.py:26: image i = b*V+v uses the planes of sample i mod B (view-major tiling)."""
    z = load_golden("tiny_v3.npz")
    B, V, D = 2, 3, int(z["d_num"])
    d_batch_0 = mvs_oracle.depth_planes(_t(z, "d_min"), _t(z, "d_int"), D)
    d_batch = torch.tile(d_batch_0, (V, 1, 1, 1))
    for i in range(B * V):
        assert torch.equal(d_batch[i], d_batch_0[i % B])
    assert not torch.equal(d_batch_0[0], d_batch_0[1])   # the fixture has distinct samples


@pytest.mark.parametrize("nv", [3, 5])
def test_float64_law_agrees_with_golden(nv):
    z = load_golden("tiny_v%d.npz" % nv)
    cv64 = mvs_oracle.cost_volume_fp64(z["feat"], z["K"], z["R"], z["T"], z["d_min"], z["d_int"],
                                       int(z["batch_size"]), nv, int(z["d_num"]))
    err = np.abs(cv64 - z["cv"]).max() / np.abs(z["cv"]).max()
    assert err < 2e-5, err


def test_soft_argmin_golden():
    z = load_golden("softargmin.npz")
    for key in ("ex", "rnd", "tie", "d5"):
        dep = mvs_oracle.extract_depth_map(_t(z, key + "_p"), _t(z, key + "_d"), int(z["n_depth_est"]))
        assert np.array_equal(dep.numpy(), z[key + "_depth"]), key
    # SURVEY §8 a7 worked example: permutation-indexed mask, not a true top-5
    assert abs(float(z["ex_depth"].ravel()[0]) - 533.636) < 1e-3


def test_cfg1_cost_volume_golden():
    from cameras import features
    z = load_golden("cfg1_cv.npz")
    B, C, D, h, w = (int(s) for s in z["shape"])
    feat = features(B * 3, C, h, w, seed=int(z["feat_seed"]))
    warped, _, _ = mvs_oracle.homography_warping(_t(z, "K"), _t(z, "R"), _t(z, "T"), _t(z, "d_min"),
                                                 _t(z, "d_int"), feat, B, 3, D, concat_growth=False)
    cv = mvs_oracle.assemble_cost_volume(warped, 3).reshape(-1)
    assert np.array_equal(cv[torch.from_numpy(z["sample_idx"])].numpy(), z["sample_val"])
    assert abs(cv.double().sum().item() - float(z["total"])) <= 1e-9 * abs(float(z["total"]))


@pytest.mark.parametrize("mode", ["eval", "train"])
def test_oracle_end_to_end_matches_reference(mode):
    """model.py:168-207 with the oracle hot path vs the reference's own forward (config 1)."""
    from weights import deterministic_state_dict
    from mvs_amd.config import MVSConfig
    from mvs_amd.model import MVSNet
    z = load_golden("cfg1_e2e.npz")
    D = int(z["d_num"])
    net = MVSNet(MVSConfig(d_num=D), device=torch.device("cpu"))
    net.load_state_dict(deterministic_state_dict(net.state_dict()))
    net.train() if mode == "train" else net.eval()
    img = torch.from_numpy(np.random.default_rng(int(z["img_seed"])).standard_normal(
        (3, 3, 512, 640), dtype=np.float32))
    with torch.no_grad():
        ini, ref, _ = mvs_oracle.mvsnet_forward(net, img, _t(z, "K"), _t(z, "R"), _t(z, "T"),
                                                _t(z, "d_min"), _t(z, "d_int"), 1, 3, D, (128, 160))
    np.testing.assert_allclose(ini.numpy(), z[mode + "_initial"], rtol=1e-6, atol=0)
    np.testing.assert_allclose(ref.numpy(), z[mode + "_refined"], rtol=1e-5, atol=1e-3)


# ---------------- analytic known answers for the kornia restatement (parity unpinned) --------
def _warp(img, H, hw):
    return kornia_warp.warp_perspective(img, H, hw, align_corners=False)


def test_identity_homography_resamples_by_w_over_w_minus_1():
    """(w-1) normalisation + align_corners=False grid_sample: ix = x*w/(w-1) - 0.5."""
    h, w = 6, 9
    img = torch.arange(h * w, dtype=torch.float32).reshape(1, 1, h, w)
    out = _warp(img, torch.eye(3).unsqueeze(0), (h, w))[0, 0].double()
    xs = np.arange(w) * w / (w - 1) - 0.5
    ys = np.arange(h) * h / (h - 1) - 0.5
    ref = mvs_oracle.sample_bilinear_zero_np(img[0].double().numpy(), *np.meshgrid(xs, ys))[0]
    np.testing.assert_allclose(out.numpy(), ref, atol=1e-4)


def test_pure_translation_samples_inverse_homography():
    h, w = 7, 10
    rng = np.random.default_rng(0)
    img = torch.from_numpy(rng.standard_normal((1, 2, h, w)).astype(np.float32))
    H = torch.tensor([[1.0, 0.0, 2.0], [0.0, 1.0, -1.0], [0.0, 0.0, 1.0]]).unsqueeze(0)
    out = _warp(img, H, (h, w))[0].double().numpy()
    gx, gy = np.meshgrid(np.arange(w, dtype=np.float64), np.arange(h, dtype=np.float64))
    ix = (gx - 2.0) * w / (w - 1) - 0.5          # source = H^-1 [x, y, 1]
    iy = (gy + 1.0) * h / (h - 1) - 0.5
    ref = mvs_oracle.sample_bilinear_zero_np(img[0].double().numpy(), ix, iy)
    np.testing.assert_allclose(out, ref, atol=1e-4)


def test_out_of_bounds_homography_gives_zeros():
    img = torch.ones(1, 3, 5, 6)
    H = torch.tensor([[1.0, 0.0, 100.0], [0.0, 1.0, 0.0], [0.0, 0.0, 1.0]]).unsqueeze(0)
    assert _warp(img, H, (5, 6)).abs().max().item() == 0.0


def test_small_homogeneous_scale_branch():
    """|s| <= 1e-8: kornia keeps (u, v) undivided (scale 1) instead of dividing by ~0."""
    pts = torch.tensor([[[0.5, -0.25, 1e-9], [0.5, -0.25, 2.0]]])
    out = kornia_warp.convert_points_from_homogeneous(pts)
    assert torch.equal(out[0, 0], torch.tensor([0.5, -0.25]))
    assert torch.allclose(out[0, 1], torch.tensor([0.25, -0.125]))


def test_reference_fp32_noise_level():
    """Pins the tolerance used by the GPU parity tests: at config 1 the reference's own fp32 cost
    volume deviates from the float64 law by ~1e-4 relative L2 at most (plane 5 shown)."""
    from cameras import features
    z = load_golden("cfg1_cv.npz")
    B, C, D, h, w = (int(s) for s in z["shape"])
    feat = features(3, C, h, w, seed=int(z["feat_seed"]))
    cams = [_t(z, k) for k in ("K", "R", "T", "d_min", "d_int")]
    k = 5
    cv64 = mvs_oracle.cost_volume_fp64(feat.numpy(), *[c.numpy() for c in cams], 1, 3, D,
                                       d_begin=k, d_count=1)
    warped, _, _ = mvs_oracle.homography_warping(*cams, feat, 1, 3, D, concat_growth=False)
    cv32 = mvs_oracle.assemble_cost_volume(warped, 3)[:, :, k:k + 1].double().numpy()
    d = np.abs(cv32 - cv64)
    rel = np.linalg.norm(d) / np.linalg.norm(cv64)
    assert 1e-5 < rel < 1.5e-4 and d.max() < 1e-3, (rel, d.max())


def test_cfg2_selfnoise_fixture_is_consistent():
    """CPU: tests/golden/cfg2_selfnoise.npz (make_cfg2_selfnoise.py) -- the recorded CPU-fp32-vs-f64
    flip and within-1e-4 fractions follow from its stored kept-plane sets and depths; kept planes are
    sorted plane indices < D; the f64 depth is finite and positive."""
    import os
    from make_cfg2_selfnoise import significant_flips
    fx = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cfg2_selfnoise.npz"))
    assert fx["keep64"].shape == fx["keep32"].shape == (4, 5, 128, 160)
    assert fx["ini64"].shape == (4, 128, 160) and np.isfinite(fx["ini64"]).all() and (fx["ini64"] > 0).all()
    for k in ("keep64", "keep32"):
        assert (np.diff(fx[k].astype(int), axis=1) > 0).all() and fx[k].max() < 192
    for b in range(4):
        flip = significant_flips(fx["keep32"][b], fx["sig32"][b].astype(np.float32), fx["keep64"][b],
                                 fx["sig64"][b].astype(np.float32))
        assert flip.mean() == fx["cpu_flip_frac"][b]
        rel = np.abs(fx["ini32"][b].astype(np.float64) - fx["ini64"][b]) / np.abs(fx["ini64"][b])
        assert (rel[~flip] <= 1e-4).mean() == fx["cpu_within_1e4_unflipped"][b]
        assert rel[~flip].max() == fx["cpu_max_rel_unflipped"][b]
    # the reference's own noise is what the GPU test is measured against: recorded, non-trivial
    assert 0 < fx["cpu_flip_frac"].max() < 0.01 and fx["cpu_within_1e4_unflipped"].min() > 0.98


def test_cfg5_oracle_fixture_is_consistent():
    """CPU: tests/golden/cfg5_oracle.npz (make_cfg5_oracle.py) -- shapes, sorted kept planes, the
    4,096 sampled voxels are the script's seeded draw, probabilities in [0, 1], depth finite."""
    import os
    from make_cfg5_oracle import sample_voxels
    fx = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cfg5_oracle.npz"))
    assert fx["ini"].shape == (296, 400) and np.isfinite(fx["ini"]).all() and (fx["ini"] > 0).all()
    assert fx["keep"].shape == fx["sig"].shape == (5, 296, 400) and fx["sig"].dtype == bool
    assert (np.diff(fx["keep"].astype(int), axis=0) > 0).all() and fx["keep"].max() < 256
    pz, py, px = sample_voxels(256, 296, 400)
    assert np.array_equal(pz, fx["pz"]) and np.array_equal(py, fx["py"]) and np.array_equal(px, fx["px"])
    assert ((fx["pv"] >= 0) & (fx["pv"] <= 1)).all() and fx["tie"].mean() < 0.01
