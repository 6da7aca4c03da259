"""GPU parity at the BASELINE.json workloads (configs[1..4]), beyond the small cases of
test_gpu_parity.py.  Every test runs the HIP path through the C ABI (mvs_amd.ops) and checks it
against the CPU oracle (oracle/mvs_oracle.py: the reference's op sequence, and its float64 law).

  cfg 2  B=4, V=3, 640x512 images (128x160 features), D=192 -- the bench workload, end to end
  cfg 3  B=8, V=5, D=192 -- every sample, 10 planes each, including the planes whose workgroups
         overflow the LDS budget and take the global-gather fallback
  cfg 4  D=256 split in 32-plane shards -- the last shard [224, 256) bit-equal to the full volume
  cfg 5  B=1, V=3, 1600x1184 images (296x400 features), D=256 -- plane spot-checks

Tolerances (as test_gpu_parity.py): cost volume vs the float64 law max|d| <= 1e-3 + 1e-3|ref| and
relative L2 <= 1e-4 (the reference's own fp32 cost volume is 5.8e-4 / 6.1e-5 from it at config 1).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _close(gpu, ref, atol=1e-3, rtol=1e-3, l2=1e-4):
    gpu = gpu.detach().double().cpu()
    ref = torch.as_tensor(np.asarray(ref)).double()
    assert gpu.shape == ref.shape, (gpu.shape, ref.shape)
    d = (gpu - ref).abs()
    bad = d > atol + rtol * ref.abs()
    assert not bad.any(), "max|d|=%g at %s (ref %g)" % (d.max(), d.argmax(), ref.reshape(-1)[d.argmax()])
    rel = d.norm() / max(ref.norm().item(), 1e-30)
    assert rel <= l2, "relative L2 error %g" % rel


def _law(feat, K, R, T, d_min, d_int, b, V, k):
    """float64 law of sample b, plane k: [1, C, 1, h, w]."""
    import mvs_oracle
    sl = slice(b * V, (b + 1) * V)
    return mvs_oracle.cost_volume_fp64(feat[sl], K[sl], R[sl], T[sl], d_min[b:b + 1], d_int[b:b + 1],
                                       1, V, k + 1, d_begin=k, d_count=1)


def test_cfg3_every_sample_including_lds_fallback_planes():
    """cfg 3 (B=8, V=5, D=192): 10 planes of every sample against the float64 law.  Planes 0-3 are
    the first plane group, whose workgroups overflow the V=5 LDS budget in samples 0-6 (the CPU
    footprint model, tests/footprint.py, asserts that here) and take the global-gather path."""
    from cameras import camera_batch, depth_range, features
    from footprint import fallback_map
    from mvs_amd import warp_and_assemble_cost_volume
    B, V, C, h, w, D = 8, 5, 32, 128, 160, 192
    K, R, T = camera_batch(B, V, h, w)
    d_min, d_int = depth_range(B)
    fb, pg = fallback_map(K, R, T, d_min, d_int, B, V, h, w, 0, 8)
    assert pg == 4 and fb[:7, 0].any(axis=(1, 2)).all(), "plane group 0 no longer overflows"
    feat = features(B * V, C, h, w, seed=33)
    with torch.no_grad():
        cv, _, _ = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, feat.to(DEV), B, V, d_num=D)
    assert torch.isfinite(cv).all() and (cv >= 0).all()
    fn = feat.numpy()
    for b in range(B):
        for k in (0, 1, 2, 3, 17, 63, 100, 150, 190, 191):
            _close(cv[b:b + 1, :, k:k + 1], _law(fn, K, R, T, d_min, d_int, b, V, k))


def test_forced_lds_fallback_matches_law():
    """A zoomed-out source camera (K x 0.25: the reference tile's taps spread 4x wider) makes about
    a tenth of the workgroups overflow LDS even with unpadded rows; every plane of both samples must
    still follow the float64 law, and the staged and fallback workgroups of one launch agree with
    each other through the law."""
    from cameras import camera_batch, depth_range, features
    from footprint import fallback_map
    from mvs_amd import warp_and_assemble_cost_volume
    B, V, C, h, w, D = 2, 3, 32, 128, 160, 32
    K, R, T = camera_batch(B, V, h, w)
    K[2::3, :2, :] *= 0.25
    d_min, d_int = depth_range(B, d_int=4.0)
    fb, _ = fallback_map(K, R, T, d_min, d_int, B, V, h, w, 0, D)
    assert 0.02 < fb.mean() < 0.5, fb.mean()
    feat = features(B * V, C, h, w, seed=44)
    with torch.no_grad():
        cv, _, _ = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, feat.to(DEV), B, V, d_num=D)
    import mvs_oracle
    ref = mvs_oracle.cost_volume_fp64(feat.numpy(), K, R, T, d_min, d_int, B, V, D)
    _close(cv, ref)


@pytest.mark.parametrize("B", [1, 4])
def test_cfg4_last_shard_bit_equal_to_full_volume(B):
    """cfg 4 (D=256 over 8 ranks, 32 planes each): each rank's shard is the kernel launched with
    d_begin/d_count; the shard [224, 256) (and [0, 32)) must equal the full volume's slice bit for
    bit (per-plane arithmetic does not depend on the launch), and follow the float64 law."""
    from cameras import camera_batch, depth_range, features
    from mvs_amd import warp_and_assemble_cost_volume
    V, C, h, w, D = 3, 32, 128, 160, 256
    K, R, T = camera_batch(B, V, h, w)
    d_min, d_int = depth_range(B)
    feat = features(B * V, C, h, w, seed=40 + B).to(DEV)
    with torch.no_grad():
        full, _, _ = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, feat, B, V, d_num=D)
        for d_begin in (224, 0):
            shard, _, _ = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, feat, B, V, d_num=D,
                                                        d_begin=d_begin, d_count=32)
            assert torch.equal(shard, full[:, :, d_begin:d_begin + 32])
    fn = feat.cpu().numpy()
    for k in (224, 240, 255):
        _close(full[:1, :, k:k + 1], _law(fn, K, R, T, d_min, d_int, 0, V, k))


def test_cfg5_full_resolution_planes():
    """cfg 5 (1600x1184 images -> 296x400 features, D=256, B=1): 8 planes against the float64 law,
    plus volume-wide properties (finite, non-negative, deterministic)."""
    from cameras import camera_batch, depth_range, features
    from mvs_amd import warp_and_assemble_cost_volume
    B, V, C, h, w, D = 1, 3, 32, 296, 400, 256
    K, R, T = camera_batch(B, V, h, w)
    d_min, d_int = depth_range(B)
    feat = features(B * V, C, h, w, seed=55)
    with torch.no_grad():
        cv, _, _ = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, feat.to(DEV), B, V, d_num=D)
        cv2, _, _ = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, feat.to(DEV), B, V, d_num=D)
    assert torch.equal(cv, cv2)
    assert torch.isfinite(cv).all() and (cv >= 0).all()
    fn = feat.numpy()
    for k in (0, 1, 31, 64, 128, 200, 254, 255):
        _close(cv[:, :, k:k + 1], _law(fn, K, R, T, d_min, d_int, 0, V, k))


def _kept_planes(P, n_est, stable=True):
    """[D,h,w] -> boolean mask of the planes depthmap.py keeps.  stable=True: ties in P ranked by
    ascending plane index (the HIP kernel's rule); stable=False: torch.sort exactly as the reference
    calls it (CPU introsort for D > 16: exact ties ordered arbitrarily)."""
    t = torch.from_numpy(np.ascontiguousarray(P))
    _, order = torch.sort(t, dim=0, descending=True, stable=stable)
    return (order < n_est).numpy()


def _stable_depth(P, d):
    """depthmap.py:4-22 with the stable tie rule, float64: P [B,1,D,h,w], d [B,D,1,1] -> [B,1,h,w]."""
    P = np.asarray(P, np.float64)
    out = np.empty((P.shape[0], 1) + P.shape[3:])
    for b in range(P.shape[0]):
        m = _kept_planes(P[b, 0].astype(np.float32), 5)
        num = (np.asarray(d, np.float64)[b].reshape(-1, 1, 1) * P[b, 0] * m).sum(0)
        out[b, 0] = num / (P[b, 0] * m).sum(0)
    return out


def _tie_pixels(P):
    """[D,h,w] -> pixels whose reference mask (torch.sort, unstable) differs from the stable rule:
    an exact tie in P at the rank-5 boundary, decided arbitrarily by the reference's sort."""
    return (_kept_planes(P, 5, stable=False) != _kept_planes(P, 5)).any(0)


def _log(msg):
    """Progress of the long end-to-end tests (a GPU run silent for minutes is taken to be hung)."""
    import time
    print("[%s] %s" % (time.strftime("%H:%M:%S"), msg), flush=True)


def _prob_diff(live, full):
    """Live-region vs full-volume probabilities: max |diff| and max relative diff where P > 1e-6."""
    d = (live - full).abs()
    big = full.abs() > 1e-6
    return {"live_vs_full_prob_max_abs": float(d.max().item()),
            "live_vs_full_prob_max_rel_p_gt_1e-6": float((d[big] / full.abs()[big]).max().item())}


def _depth_parity(P_gpu, P_ref, d_gpu, d_ref):
    """Mask flips and relative depth error of one sample: P [D, h, w], depth [h, w] (numpy).  A
    pixel counts as flipped when the two P give different masks, or when the reference's own
    (unstable-sort) mask is tie-ambiguous there."""
    flip = (_kept_planes(P_gpu, 5) != _kept_planes(P_ref, 5)).any(0) | _tie_pixels(P_ref)
    rel = np.abs(d_gpu - d_ref) / np.abs(d_ref)
    return flip, rel


def _flip_quantiles(rel, flip):
    """Relative depth error on the mask-flipped pixels: p50 / p99 / max, their count (0s when none) and
    the largest ones in descending order ("top", at most 256: the order statistics the criterion uses)."""
    r = rel[flip]
    if r.size == 0:
        return {"n": 0, "p50": 0.0, "p99": 0.0, "max": 0.0, "top": []}
    return {"n": int(r.size), "p50": float(np.quantile(r, 0.5)), "p99": float(np.quantile(r, 0.99)),
            "max": float(r.max()), "top": [float(v) for v in np.sort(r)[::-1][:256]]}


def _reference_flip_quantiles_cfg2(with_rel=False):
    """The reference's OWN flipped-pixel error at cfg 2, per sample: its fp32 depth (the CPU fp32 oracle)
    against the float64 law on the pixels where the two masks differ in a weight-carrying plane
    (tests/golden/cfg2_selfnoise.npz, make_cfg2_selfnoise.py)."""
    import os
    from make_cfg2_selfnoise import significant_flips
    fx = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cfg2_selfnoise.npz"))
    out, rels = [], []
    for b in range(fx["ini64"].shape[0]):
        cflip = significant_flips(fx["keep32"][b], fx["sig32"][b].astype(np.float32), fx["keep64"][b],
                                  fx["sig64"][b].astype(np.float32))
        crel = np.abs(fx["ini32"][b].astype(np.float64) - fx["ini64"][b]) / np.abs(fx["ini64"][b])
        out.append(_flip_quantiles(crel, cflip))
        rels.append(crel)
    return (out, rels) if with_rel else out


TAIL_T = (1e-4, 1e-3, 1e-2, 5e-2)


def _tail_fracs(rel):
    """Share of ALL pixels whose relative depth error exceeds each threshold of TAIL_T."""
    return [float((rel > t).mean()) for t in TAIL_T]


def _flips_within_reference(gq, rq, g_rel, r_rel, what):
    """Every pixel of the map under the reference's own noise, against one yardstick
    (the float64 law at cfg 2, the fp64-matrix fixture at cfg 5):
      * the flipped pixels, by order statistics: the GPU's k-th largest flipped-pixel error no larger than
        the reference's own k-th largest on ITS flips, for every k up to the GPU's flip count (which
        includes max and, for the GPU's own count, its p99) -- and no more GPU flips than the reference's
        beyond that;
      * the whole map: for every threshold t of TAIL_T (1e-4 ... 5e-2) the share of pixels off by more
        than t no larger for the GPU than for the reference -- flipped and unflipped pixels alike.
    Quantiles of the two flip sets are recorded, not compared: the GPU flips 4-40x fewer pixels than the
    reference (39 against 159 at cfg 2, 66 against 2,648 at cfg 5, r6d), so a p99 of 66 values is their
    second largest, against the 27th largest of 2,648 (r6w: 0.083 against 0.077 at cfg 5 while the GPU's
    largest, 0.084, is half the reference's 0.158).  A flip's error is the depth jump of swapping two
    near-tied planes -- a property of the network's probabilities (GPU 0.52 % / 0.61 %, reference 0.49 % /
    0.55 % at the median)."""
    g_top, r_top = gq.get("top", []), rq.get("top", [])
    assert len(g_top) <= len(r_top) or gq["n"] <= rq["n"], (what, "more flips than the reference", gq["n"], rq["n"])
    for k, v in enumerate(g_top[:len(r_top)]):
        assert v <= r_top[k], (what, "k-th largest flipped-pixel error", k, v, r_top[k], gq["n"], rq["n"])
    gt, rt = _tail_fracs(g_rel), _tail_fracs(r_rel)
    assert all(a <= b for a, b in zip(gt, rt)), (what, "tail shares", dict(zip(TAIL_T, gt)), dict(zip(TAIL_T, rt)))


@pytest.mark.parametrize("arithmetic", ["fp32", "split_f16"])
def test_cfg2_end_to_end_as_benchmarked(arithmetic):
    """The bench workload exactly as bench.py runs it: B=4, V=3, 640x512, D=192, BN eval mode,
    no_grad, MVSNet.forward in the bench's arithmetic -- "fp32" (the headline: fp32 channel-quad cost
    volume -> exact-fp32 live-region regulariser: depth-Winograd VALU conv_0_0, fp32-MFMA region convs) or
    the "split_f16" opt-in (split cost volume -> split head -> split-fp16 region convs) -> HIP softmax /
    soft-argmin -> refinement.

      * the benchmarked call's OWN probability volume (captured from the regulariser by a forward
        hook) against the CPU oracle forward (oracle/mvs_oracle.py::mvsnet_forward, the reference's
        full op sequence, one sample at a time): 2e-3 relative, recorded per sample; and bit-equal to
        the regulariser fed that arithmetic's materialised volume directly;
      * that P against CostVolumeReg.forward_full (the reference's op sequence on MIOpen) on the same
        GPU, every voxel of all 4 samples: 1e-4 relative;
      * depth: 1e-4 relative on >= 99.95 % of the pixels whose permutation mask is the same under both
        P, mask flips < 2 %; the measured fractions are recorded (conftest.record_parity);
      * the flipped pixels: their relative depth error against the oracle (p50 / p99 / max, on the
        pixels whose masks differ in a weight-carrying plane) recorded beside the reference's own fp32
        error against the float64 law on ITS flipped pixels (cfg2_selfnoise.npz); asserted in
        test_cfg2_depth_flips_within_reference_self_noise against the same yardstick;
      * refined depth of all 4 samples against the CPU refinement of the GPU's initial depth.
    """
    import mvs_oracle
    from cameras import camera_batch, depth_range
    from conftest import record_parity
    from make_cfg2_selfnoise import kept_with_p, significant_flips
    from weights import deterministic_state_dict
    from mvs_amd import warp_and_assemble_cost_volume, extract_depth_map
    from mvs_amd.config import MVSConfig
    from mvs_amd.model import MVSNet
    B, V, D, H, W = 4, 3, 192, 512, 640
    net = MVSNet(MVSConfig(d_num=D, in_h=H, in_w=W, arithmetic=arithmetic), device=torch.device("cpu"))
    net.load_state_dict(deterministic_state_dict(net.state_dict()))
    net.eval()
    K, R, T = camera_batch(B, V, H // 4, W // 4)
    d_min, d_int = depth_range(B)
    img = torch.randn(B * V, 3, H, W, generator=torch.Generator().manual_seed(1000))
    cpu = _cfg2_cpu_oracle(net, img, K, R, T, d_min, d_int)
    with torch.no_grad():
        _log("cfg2 %s: GPU forward (live) and forward_full" % arithmetic)
        g = net.to(DEV)
        g_img = img.to(DEV)
        heads = []
        hook = g.cost_volume_reg.register_forward_hook(lambda m, i, o: heads.append(o.detach()))
        try:
            g_ini_full, g_ref = g(g_img, K, R, T, d_min, d_int, B, V)      # the benchmarked call
        finally:
            hook.remove()
        assert len(heads) == 1
        p_head = heads[0]
        feats = g.feature_encoder(g_img)
        # the benchmarked regulariser input, materialised: the fp32 channel-quad volume (fp32) or the split
        # volume (split_f16); the NCDHW volume of the same values feeds forward_full
        cv4, d_batch, _ = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, feats, B, V, d_num=D,
                                                        channel_quads=True, split=arithmetic == "split_f16")
        assert g.cost_volume_reg.live_region
        g_prob = g.cost_volume_reg(cv4)
        del cv4
        g_ini = extract_depth_map(g_prob, d_batch)
        cv, _, _ = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, feats, B, V, d_num=D)
        prob_full = g.cost_volume_reg.forward_full(cv)
        del cv
    ref_q = _reference_flip_quantiles_cfg2()
    flips, within, within_unflipped, worst, p_rel, p_rel_head, fq = [], [], [], [], [], [], []
    for b in range(B):
        c_ini, Pc = cpu[b]
        Pg = g_prob[b, 0].cpu().numpy()
        p_rel.append(float((np.abs(Pg - Pc) / np.maximum(np.abs(Pc), 1e-8 / 2e-3)).max()))
        Ph = p_head[b, 0].cpu().numpy()
        p_rel_head.append(float((np.abs(Ph - Pc) / np.maximum(np.abs(Pc), 1e-8 / 2e-3)).max()))
        flip, rel = _depth_parity(Pg, Pc, g_ini_full[b, 0].cpu().numpy(), c_ini)
        flips.append(float(flip.mean()))
        within.append(float((rel <= 1e-4).mean()))
        within_unflipped.append(float((rel[~flip] <= 1e-4).mean()))
        worst.append(float(rel[~flip].max()))
        (kg, qg), (kc, qc) = kept_with_p(Pg), kept_with_p(Pc)
        fq.append(dict(significant=_flip_quantiles(rel, significant_flips(kg, qg, kc, qc)),
                       all_flipped=_flip_quantiles(rel, flip)))
    # the measured numbers first (recorded even when an assertion below fails)
    record_parity("cfg2_e2e_vs_cpu_oracle" + ("" if arithmetic == "fp32" else "_split_f16"), samples=B,
                  arithmetic=arithmetic, mask_flip_frac=flips, within_1e4_frac=within,
                  within_1e4_frac_unflipped=within_unflipped, max_rel_unflipped=worst,
                  flipped_pixel_rel_error_vs_cpu_oracle=fq,
                  reference_fp32_vs_float64_flipped_pixel_rel_error=ref_q,
                  prob_max_rel_vs_cpu=p_rel, benchmarked_prob_max_rel_vs_cpu=p_rel_head,
                  benchmarked_prob_bit_equal_to_materialised_path=bool(torch.equal(p_head, g_prob)),
                  **_prob_diff(g_prob, prob_full))
    for b in range(B):   # the benchmarked path's own P against the oracle (named before the equality)
        np.testing.assert_allclose(p_head[b, 0].cpu().numpy(), cpu[b][1], rtol=2e-3, atol=1e-8)
    assert torch.equal(p_head, g_prob)
    assert torch.equal(g_ini, g_ini_full)
    torch.testing.assert_close(g_prob, prob_full, rtol=1e-4, atol=1e-9)
    for b in range(B):
        np.testing.assert_allclose(g_prob[b, 0].cpu().numpy(), cpu[b][1], rtol=2e-3, atol=1e-8)
        assert flips[b] < 0.02, "sample %d: %.2f %% of pixels change their mask" % (b, 100 * flips[b])
        assert within_unflipped[b] >= 1 - 5e-4, "sample %d: %.4f of unflipped pixels within 1e-4" % (
            b, within_unflipped[b])
        assert worst[b] <= 1e-2, worst[b]
    # refinement (model.py:189-205) isolated: the CPU refine net applied to the GPU's own initial
    # depth must give the GPU's refined depth (the random-weight refine net amplifies initial-depth
    # differences ~1e3x at D=192, so comparing against the oracle's refined depth would test the
    # soft-argmin mask flips again); relative to max(|depth|, 100 mm)
    with torch.no_grad():
        net_cpu = net.to(torch.device("cpu"))
        c_ref_on_g = net_cpu.refine(img, g_ini_full.cpu(), d_min, d_int, torch.arange(0, B * V, V))
    gr, cr = g_ref.cpu().numpy(), c_ref_on_g.numpy()
    rel_r = np.abs(gr - cr) / np.maximum(np.abs(cr), 100.0)
    assert rel_r.max() <= 1e-4, rel_r.max()


_CFG2_CPU = {}


def _cfg2_cpu_oracle(net, img, K, R, T, d_min, d_int):
    """The CPU oracle forward of the 4 cfg-2 samples [(initial depth, P)], computed once per process
    (both arithmetic cases of test_cfg2_end_to_end_as_benchmarked compare with it)."""
    import mvs_oracle
    if "cpu" not in _CFG2_CPU:
        B, V, D, H, W = 4, 3, 192, 512, 640
        cpu = []
        with torch.no_grad():
            for b in range(B):
                _log("cfg2: CPU oracle forward of sample %d" % b)
                sl = slice(b * V, (b + 1) * V)
                c_ini, _, c_prob = mvs_oracle.mvsnet_forward(net, img[sl], K[sl], R[sl], T[sl], d_min[b:b + 1],
                                                             d_int[b:b + 1], 1, V, D, (H // 4, W // 4))
                cpu.append((c_ini[0, 0].numpy(), c_prob[0, 0].numpy()))
        _CFG2_CPU["cpu"] = cpu
    return _CFG2_CPU["cpu"]


def test_cfg2_depth_flips_within_reference_self_noise():
    """cfg 2's depth against the float64 law, with the reference's OWN fp32 noise as the yardstick
    (tests/golden/make_cfg2_selfnoise.py: the CPU fp32 oracle and mvs_oracle.mvsnet_forward64 on the
    same weights / images, committed).  The benchmarked call (MVSNet.forward in the default fp32 arithmetic:
    fp32 cost volume, exact-fp32 regulariser, HIP soft-argmin) is run on all 4 samples; with its probability
    volume (the regulariser's output, captured by a forward hook):

      * GPU-vs-f64 mask flips (the depthmap.py:11-15 kept-plane sets differ in a plane that carries
        weight, P >= 1e-7: swaps among the fp32 softmax's exact zeros move no depth) <= 1.5 x the
        CPU fp32 oracle's own flips against f64 (+ 0.05 % of the pixels, for samples where the CPU
        flips on almost none: sample 0 flips 0.04 %), per sample;
      * on the pixels unflipped against f64: the fraction within 1e-4 relative of the f64 depth is no
        worse than the CPU oracle's own (99.17-99.32 %) by more than 0.1 percentage point, and the
        99.9th percentile of the relative error <= 1.5 x the CPU oracle's (the f64 law is free of the
        reference's fp32 homography rounding, so "every unflipped pixel within 1e-4" does not hold
        for the reference itself: its worst unflipped pixels are 5-10 % off, the GPU's 2-27 % --
        single pixels whose near-tied planes the random-weight softmax re-weights, recorded, not
        asserted);
      * on the pixels flipped against f64: the GPU's relative depth error (p50 / p99 / max) no larger
        than the CPU oracle's own on its flipped pixels (every pixel of the map is
        then under a criterion)."""
    import os
    from conftest import record_parity
    from make_cfg2_selfnoise import GEOM, cfg2_inputs, kept_with_p, significant_flips
    fx = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cfg2_selfnoise.npz"))
    B, V, D, H, W = GEOM
    net, img, K, R, T, d_min, d_int = cfg2_inputs()
    g = net.to(DEV)
    probs = []
    hook = g.cost_volume_reg.register_forward_hook(lambda m, i, o: probs.append(o.detach()))
    try:
        with torch.no_grad():
            ini, _ = g(img.to(DEV), K, R, T, d_min, d_int, B, V)
    finally:
        hook.remove()
    assert len(probs) == 1
    P = probs[0].cpu().numpy()
    ini = ini.cpu().numpy()
    flips, within, worst, q999, cpu_q999, worst_px = [], [], [], [], [], []
    for b in range(B):
        kg, pg = kept_with_p(P[b, 0])
        flip = significant_flips(kg, pg, fx["keep64"][b], fx["sig64"][b].astype(np.float32))
        rel = np.abs(ini[b, 0].astype(np.float64) - fx["ini64"][b]) / np.abs(fx["ini64"][b])
        flips.append(float(flip.mean()))
        within.append(float((rel[~flip] <= 1e-4).mean()))
        worst.append(float(rel[~flip].max()))
        # the worst unflipped pixel, for the record: where it is, the GPU's 8 most probable planes
        # there, the kept planes of both, and the three depths (DESIGN.md §4 analyses it)
        yx = np.unravel_index(np.argmax(np.where(flip, -1.0, rel)), rel.shape)
        top = np.argsort(-P[b, 0][:, yx[0], yx[1]], kind="stable")[:8]
        worst_px.append(dict(y=int(yx[0]), x=int(yx[1]), gpu_top8_planes=top.tolist(),
                             gpu_top8_p=P[b, 0][top, yx[0], yx[1]].tolist(),
                             gpu_kept=kg[:, yx[0], yx[1]].tolist(), f64_kept=fx["keep64"][b][:, yx[0], yx[1]].tolist(),
                             fp32_ref_kept=fx["keep32"][b][:, yx[0], yx[1]].tolist(),
                             depth_gpu=float(ini[b, 0][yx]), depth_f64=float(fx["ini64"][b][yx]),
                             depth_fp32_ref=float(fx["ini32"][b][yx])))
        q999.append(float(np.quantile(rel[~flip], 0.999)))
        cflip = significant_flips(fx["keep32"][b], fx["sig32"][b].astype(np.float32), fx["keep64"][b],
                                  fx["sig64"][b].astype(np.float32))
        crel = np.abs(fx["ini32"][b].astype(np.float64) - fx["ini64"][b]) / np.abs(fx["ini64"][b])
        cpu_q999.append(float(np.quantile(crel[~cflip], 0.999)))
    cpu_flip, cpu_within, cpu_worst = (fx["cpu_flip_frac"], fx["cpu_within_1e4_unflipped"],
                                       fx["cpu_max_rel_unflipped"])
    # the flipped pixels: the GPU's relative depth error against f64 on its flips, beside the reference's own
    # on its flips (with this every pixel of the map is under a criterion)
    gq, grel = [], []
    rq, rrel = _reference_flip_quantiles_cfg2(with_rel=True)
    for b in range(B):
        kg, pg = kept_with_p(P[b, 0])
        flip = significant_flips(kg, pg, fx["keep64"][b], fx["sig64"][b].astype(np.float32))
        rel = np.abs(ini[b, 0].astype(np.float64) - fx["ini64"][b]) / np.abs(fx["ini64"][b])
        gq.append(_flip_quantiles(rel, flip))
        grel.append(rel)
    record_parity("cfg2_vs_float64_law", samples=B, gpu_flip_frac=flips, cpu_fp32_flip_frac=cpu_flip.tolist(),
                  gpu_within_1e4_unflipped=within, cpu_fp32_within_1e4_unflipped=cpu_within.tolist(),
                  gpu_q999_rel_unflipped=q999, cpu_fp32_q999_rel_unflipped=cpu_q999,
                  gpu_max_rel_unflipped=worst, cpu_fp32_max_rel_unflipped=cpu_worst.tolist(),
                  gpu_worst_unflipped_pixel=worst_px, gpu_flipped_pixel_rel_error=gq,
                  cpu_fp32_flipped_pixel_rel_error=rq, tail_thresholds=list(TAIL_T),
                  gpu_tail_share_all_pixels=[_tail_fracs(r) for r in grel],
                  cpu_fp32_tail_share_all_pixels=[_tail_fracs(r) for r in rrel])
    for b in range(B):
        assert flips[b] <= 1.5 * cpu_flip[b] + 5e-4, (b, flips[b], cpu_flip[b])
        _flips_within_reference(gq[b], rq[b], grel[b], rrel[b], "cfg2 sample %d vs f64" % b)
        assert within[b] >= cpu_within[b] - 1e-3, (b, within[b], cpu_within[b])
        assert q999[b] <= 1.5 * cpu_q999[b], (b, q999[b], cpu_q999[b])


E2E_CFGS = {   # BASELINE.json configs[2] and configs[4]: (B, V, D, image H, image W)
    "cfg3": (8, 5, 192, 512, 640),
    "cfg5": (1, 3, 256, 1184, 1600),
}


@pytest.mark.parametrize("cfg", sorted(E2E_CFGS))
def test_model_end_to_end_at_cfg3_cfg5(cfg):
    """MVSNet.forward end to end at cfg 3 (B=8, V=5, 640x512, D=192) and cfg 5 (B=1, V=3, 1600x1184
    full-resolution images -> 296x400 features, D=256), BN eval, no_grad, as bench.py's e2e_configs
    times it:
      * the benchmarked call (fp32 channel-quad cost volume -> live-region HIP regulariser in exact fp32)
        gives the same initial depth as that regulariser path called directly;
      * live-path probabilities against CostVolumeReg.forward_full (the reference's op sequence,
        model.py:100-126, on MIOpen) on every voxel of every sample: 1e-4 relative;
      * the HIP soft-argmin on that P against the oracle's extract_depth_map (depthmap.py:4-22,
        torch.sort on the CPU): 1e-5 relative;
      * the depth of the reference op sequence (forward_full's P through the oracle soft-argmin)
        against the benchmarked depth: mask flips < 2 %, >= 99.95 % of the unflipped pixels within
        1e-4 relative; both fractions recorded (conftest.record_parity)."""
    import mvs_oracle
    from cameras import camera_batch, depth_range
    from conftest import record_parity
    from weights import deterministic_state_dict
    from mvs_amd import warp_and_assemble_cost_volume, extract_depth_map
    from mvs_amd.config import MVSConfig
    from mvs_amd.model import MVSNet
    B, V, D, H, W = E2E_CFGS[cfg]
    net = MVSNet(MVSConfig(d_num=D, in_h=H, in_w=W), device=torch.device("cpu"))
    net.load_state_dict(deterministic_state_dict(net.state_dict()))
    g = net.to(DEV).eval()
    K, R, T = camera_batch(B, V, H // 4, W // 4)
    d_min, d_int = depth_range(B)
    img = torch.randn(B * V, 3, H, W, generator=torch.Generator().manual_seed(2000 + B)).to(DEV)
    _log("%s: GPU forward (live)" % cfg)
    with torch.no_grad():
        ini, ref = g(img, K, R, T, d_min, d_int, B, V)                 # the benchmarked call
        # the benchmarked regulariser input (the fp32 channel-quad volume: exact-fp32 regulariser)
        cv, d_batch, _ = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, g.feature_encoder(img),
                                                       B, V, d_num=D, channel_quads=True)
        P_live = g.cost_volume_reg(cv)
        del cv
        cv = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, g.feature_encoder(img), B, V, d_num=D)[0]
        if cfg == "cfg5":
            # MIOpen has only slow solvers for several cfg-5 shapes (forward_full's conv_3_0 ~10 s per
            # call; forward_live's torch branch ~7 minutes in all): the reference sequence here is
            # forward_live's PyTorch branch with every Conv3d / ConvTranspose3d as one fp32 rocBLAS
            # GEMM per tap (tests/tap_conv.py) -- independent of the HIP kernels and of MIOpen
            # (forward_live == forward_full is pinned on the CPU at 8 geometries,
            # tests/test_regulariser_live.py, and on the GPU at cfg 1-3)
            from tap_conv import tap_convs
            ref_kind = "forward_live torch branch, convs as per-tap fp32 GEMMs (tests/tap_conv.py)"
            _log("%s: forward_live torch branch (tap GEMMs)" % cfg)
            with tap_convs():
                P_full = g.cost_volume_reg.forward_live_torch(cv)
        else:
            ref_kind = "forward_full (MIOpen, model.py:100-126 op sequence)"
            _log("%s: forward_full (MIOpen)" % cfg)
            P_full = g.cost_volume_reg.forward_full(cv)
        del cv
        ini_live = extract_depth_map(P_live, d_batch)
    torch.cuda.synchronize()
    _log("%s: oracle soft-argmin (CPU)" % cfg)
    Pl, Pf, db = P_live.cpu(), P_full.cpu(), d_batch.cpu()
    d_live_oracle = mvs_oracle.extract_depth_map(Pl, db).numpy()
    d_live_stable = _stable_depth(Pl.numpy(), db.numpy())
    ties = np.stack([_tie_pixels(Pl[b, 0].numpy()) for b in range(B)])[:, None]
    d_ref = mvs_oracle.extract_depth_map(Pf, db).numpy()
    flips, within, within_unflipped = [], [], []
    for b in range(B):
        flip, rel = _depth_parity(Pl[b, 0].numpy(), Pf[b, 0].numpy(), ini[b, 0].cpu().numpy(), d_ref[b, 0])
        flips.append(float(flip.mean()))
        within.append(float((rel <= 1e-4).mean()))
        within_unflipped.append(float((rel[~flip] <= 1e-4).mean()))
    g_ini = ini.cpu().numpy()
    sa_rel = np.abs(g_ini - d_live_oracle) / np.abs(d_live_oracle)
    record_parity("%s_e2e_live_vs_reference_sequence" % cfg, B=B, V=V, D=D, image_hw=[H, W],
                  reference=ref_kind, mask_flip_frac=flips, within_1e4_frac=within,
                  within_1e4_frac_unflipped=within_unflipped, tie_pixel_frac=float(ties.mean()),
                  soft_argmin_vs_oracle_max_rel_untied=float(sa_rel[~ties].max()),
                  **_prob_diff(P_live, P_full))
    if cfg == "cfg5":
        # and against the CPU fp32 ORACLE itself, two fixtures (tests/golden/make_cfg5_oracle.py: the
        # oracle forward homography_warping -> assemble_cost_volume -> forward_full -> extract_depth_map
        # on the CPU in fp32, committed):
        #   cfg5_oracle.npz      the reference exactly (fp32 homography, homography.py:40-75 + kornia's
        #                        normalize / inverse);
        #   cfg5_oracle_h64.npz  the same ops with the sampling matrices composed in float64 and rounded
        #                        once to fp32 -- the matrices the HIP prologue forms.  Everything after
        #                        them is the reference's fp32 arithmetic, which the HIP warp + variance
        #                        reproduces bit for bit (test_gpu_parity.py::
        #                        test_cost_volume_bit_exact_vs_oracle_given_matrices).
        # Mask flips are counted on weight-carrying planes (P >= 1e-7) plus tie-ambiguous oracle pixels.
        import os
        from make_cfg2_selfnoise import kept_with_p, significant_flips
        gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
        kg, pgv = kept_with_p(Pl[0, 0].numpy())
        res = {}
        for name in ("cfg5_oracle", "cfg5_oracle_h64"):
            fx = np.load(os.path.join(gold, name + ".npz"))
            flip_o = significant_flips(kg, pgv, fx["keep"], fx["sig"].astype(np.float32)) | fx["tie"]
            d_o = fx["ini"].astype(np.float64)
            rel_o = np.abs(g_ini[0, 0].astype(np.float64) - d_o) / np.abs(d_o)
            pv = Pl[0, 0].numpy()[fx["pz"].astype(np.int64), fx["py"].astype(np.int64), fx["px"].astype(np.int64)]
            p_rel = np.abs(pv - fx["pv"]) / np.maximum(np.abs(fx["pv"]), 1e-8 / 2e-3)
            res[name] = dict(mask_flip_frac=float(flip_o.mean()),
                             within_1e4_frac_unflipped=float((rel_o[~flip_o] <= 1e-4).mean()),
                             max_rel_unflipped=float(rel_o[~flip_o].max()), sampled_p_max_rel=float(p_rel.max()),
                             oracle_tie_pixel_frac=float(fx["tie"].mean()),
                             flipped_pixel_rel_error=_flip_quantiles(rel_o, flip_o))
            if name == "cfg5_oracle_h64":
                # the reference's OWN distance from this fixture: its fp32 homography alone -- flips, and the
                # relative depth error on its flipped pixels (the two fixtures' depths and kept planes)
                fr = np.load(os.path.join(gold, "cfg5_oracle.npz"))
                flip_r = significant_flips(fr["keep"], fr["sig"].astype(np.float32), fx["keep"],
                                           fx["sig"].astype(np.float32)) | fr["tie"] | fx["tie"]
                rel_r = np.abs(fr["ini"].astype(np.float64) - d_o) / np.abs(d_o)
                rels = (rel_o, rel_r)
                res["tail_share_all_pixels"] = dict(thresholds=list(TAIL_T), gpu_vs_h64=_tail_fracs(rel_o),
                                                    reference_vs_h64=_tail_fracs(rel_r))
                res["reference_vs_h64"] = dict(mask_flip_frac=float(fx["ref_vs_h64_flip_frac"]),
                                               within_1e4_frac_unflipped=float(fx["ref_vs_h64_within_1e4_unflipped"]),
                                               max_rel_unflipped=float(fx["ref_vs_h64_max_rel_unflipped"]),
                                               flipped_pixel_rel_error=_flip_quantiles(rel_r, flip_r))
            np.testing.assert_allclose(pv, fx["pv"], rtol=2e-3, atol=1e-8)
        record_parity("cfg5_e2e_vs_cpu_oracle", vs_reference=res["cfg5_oracle"],
                      vs_reference_with_fp64_homography=res["cfg5_oracle_h64"],
                      reference_vs_reference_with_fp64_homography=res["reference_vs_h64"],
                      tail_share_all_pixels=res["tail_share_all_pixels"])
        # north_star's 1e-4 on the depth map, against the reference arithmetic given the same matrices
        h64 = res["cfg5_oracle_h64"]
        assert h64["mask_flip_frac"] < 0.02 and h64["within_1e4_frac_unflipped"] >= 0.9995, h64
        # against the reference itself: north_star's 1e-4 on every unflipped pixel's depth, and mask flips
        # no more frequent than the reference's own fp32 homography makes them against the fp64-matrix
        # fixture (r05 with the reference's permutation-indexed mask: reference vs h64 2.24 % flips, every
        # unflipped pixel within 1e-4, max 5.9e-5; GPU vs reference 2.23 %, max 5.9e-5)
        rf, own = res["cfg5_oracle"], res["reference_vs_h64"]
        assert rf["within_1e4_frac_unflipped"] >= 0.9995, rf
        assert rf["mask_flip_frac"] <= own["mask_flip_frac"] + 2e-3, (rf, own)
        # the flipped pixels: the GPU's depth error on its flips against the fp64-matrix
        # fixture no larger than the reference's own error on ITS flips against that fixture (p99 / max), and
        # the whole map's error tail no heavier than the reference's (_flips_within_reference)
        _flips_within_reference(h64["flipped_pixel_rel_error"], own["flipped_pixel_rel_error"], rels[0], rels[1],
                                "cfg5 vs h64")
    assert torch.isfinite(ini).all() and torch.isfinite(ref).all()
    assert torch.equal(ini_live, ini)
    torch.testing.assert_close(P_live, P_full, rtol=1e-4, atol=1e-9)
    # the HIP soft-argmin on the live P: the oracle's (torch.sort) depth wherever the reference's mask
    # is not tie-ambiguous, and the stable-rule float64 depth everywhere
    assert ties.mean() < 1e-3, ties.mean()
    np.testing.assert_allclose(g_ini[~ties], d_live_oracle[~ties], rtol=1e-5, atol=0)
    np.testing.assert_allclose(g_ini, d_live_stable, rtol=1e-5, atol=0)
    assert max(flips) < 0.02 and min(within_unflipped) >= 0.9995, (flips, within_unflipped)
