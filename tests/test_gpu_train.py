"""The train.py step through the drop-in (train.py:97-104): MVSNet.forward with autograd in train
mode (BatchNorm batch statistics), loss_fcn (loss.py:4-41), loss.backward(), optimizer step -- on the
GPU, against the oracle model's CPU autograd.

The GPU step runs the HIP cost volume forward (mvs::cost_volume) and its backward
(mvs::cost_volume_backward), the HIP soft-argmin with its autograd formula, and PyTorch-ROCm (MIOpen)
for the convolutions.  Three copies of the same deterministic weights (tests/golden/weights.py):

  gpu   the product path on cuda:0 (fp32);
  cpu   the oracle's reference op sequence on the CPU (fp32, oracle/mvs_oracle.py::mvsnet_forward):
        the reference's own numerics;
  law   the same model in float64 with the float64 cost-volume law (mvs_oracle.mvsnet_forward64).

Tolerances are scaled from the reference's own fp32 error: for every parameter, the relative L2
distance of the GPU gradient to the float64 gradient must be no larger than 3x the fp32 CPU
gradient's (+ 1e-4).  Both fp32 paths differ from float64 mostly through the soft-argmin's
permutation mask (depthmap.py:11-15, discontinuous in P): a pixel whose mask flips changes its
d depth / d P terms, and train-mode BatchNorm (flat P) makes such flips common, so the CPU's own
error is the scale.  BatchNorm running statistics after the step: no further from float64 than the CPU's (x 3).
"""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _rel(a, ref):
    ref = ref.double()
    n = ref.norm().item()
    return (a.double() - ref).norm().item() / max(n, 1e-30)


def test_train_step_gradients_match_oracle_autograd():
    """The GPU step against the CPU oracle's, precomputed by tests/golden/make_train_step.py (the two
    CPU autograd runs take ~4 minutes; the fixture holds the float64-law gradients / buffers and the
    fp32 CPU run's distance to them)."""
    import mvs_oracle
    from conftest import load_golden, record_parity
    from make_train_step import GEOM, train_step_inputs
    B, V, D, H, W = GEOM
    gold = load_golden("train_step_cfg1.npz")
    net, img, K, R, T, d_min, d_int, gt = train_step_inputs()
    net_g = copy.deepcopy(net).to(DEV)

    print("train step: GPU", flush=True)
    ini_g, ref_g = net_g(img.to(DEV), K, R, T, d_min, d_int, B, V)
    loss_g, acc1_g, acc2_g = mvs_oracle.loss_fcn(gt.to(DEV), ini_g, ref_g)
    loss_g.backward()
    torch.cuda.synchronize()

    lg, lc, ld = loss_g.item(), float(gold["loss_cpu_fp32"]), float(gold["loss_f64"])
    pg = dict(net_g.named_parameters())
    names = sorted(k[4:] for k in gold.files if k.startswith("g64/"))
    assert set(pg) == set(names) and len(pg) > 0
    assert all(pg[n].grad is not None for n in names)
    worst = {n: (_rel(pg[n].grad.cpu(), torch.from_numpy(gold["g64/" + n])), float(gold["ec/" + n]))
             for n in names}
    record_parity("train_step_cfg1_grads", loss_gpu=lg, loss_cpu_fp32=lc, loss_f64=ld,
                  grad_rel_l2_gpu_vs_f64_max=max(v[0] for v in worst.values()),
                  grad_rel_l2_cpu_vs_f64_max=max(v[1] for v in worst.values()),
                  per_parameter={k: [float(a), float(b)] for k, (a, b) in worst.items()})
    assert np.isfinite(lg) and abs(lg - ld) <= 3 * abs(lc - ld) + 1e-4 * abs(ld), (lg, lc, ld)
    for name, (e_g, e_c) in worst.items():
        assert torch.isfinite(pg[name].grad).all(), name
        assert e_g <= 3.0 * e_c + 1e-4, "%s: GPU grad %.3g from float64, CPU fp32 %.3g" % (name, e_g, e_c)
    # the feature encoder's gradient flows back through the HIP cost-volume backward
    assert any(n.startswith("feature_encoder") and pg[n].grad.abs().max() > 0 for n in pg)

    # BatchNorm running statistics after the step: the regulariser's and the encoder's are fed by the
    # cost volume / images (fp32 noise only); the refinement's see the initial depth, whose flipped
    # pixels differ between any two fp32 paths -- every buffer no further from float64 than the CPU
    # fp32 reference's (x 3), with a floor of 2e-6 relative: a blocked / pairwise fp32 sum of n terms
    # is within ~log2(n) * 2^-24 of float64 (n <= 10^7 here: 23 * 6e-8 = 1.4e-6), and the GPU's batch
    # statistics sum in another order than the CPU's, whose error on a given buffer may happen to be
    # 1e-7; the measured distances are recorded (PARITY train_step_bn_buffers)
    bg = dict(net_g.named_buffers())
    bufs = sorted(k[4:] for k in gold.files if k.startswith("b64/"))
    assert set(bufs) == set(bg)
    dist = {}
    for name in bufs:
        ref = torch.from_numpy(gold["b64/" + name])
        if not name.endswith("num_batches_tracked"):
            dist[name] = [_rel(bg[name].cpu(), ref), float(gold["ecb/" + name])]
    from conftest import record_parity
    record_parity("train_step_bn_buffers", gpu_vs_cpu_fp32_rel_to_f64=dist)
    for name in bufs:
        ref = torch.from_numpy(gold["b64/" + name])
        if name.endswith("num_batches_tracked"):
            assert torch.equal(bg[name].cpu(), ref), name
            continue
        e_g, e_c = dist[name]
        assert e_g <= 3.0 * e_c + 2e-6, "%s: GPU %.3g from float64, CPU fp32 %.3g" % (name, e_g, e_c)

    # one Adam step (train.py:104, Adam(model.parameters, lr) with the reference's list attribute)
    opt = torch.optim.Adam(net_g.parameters, lr=1e-3)
    before = {n: p.detach().clone() for n, p in pg.items()}
    opt.step()
    assert all(not torch.equal(before[n], pg[n].detach()) for n in pg if pg[n].grad.abs().max() > 0)


def test_train_mode_autograd_chain_smooth_loss():
    """The same autograd chain without the soft-argmin's discontinuous mask: a smooth loss on the
    probability volume, L = sum(P * Wr), through the train-mode regulariser (MIOpen), the HIP cost
    volume backward and the encoder, B=2 with distinct depth ranges (the i mod B plane tiling), at a
    reduced geometry (256x320 images, D=16).  Every parameter's gradient: relative L2 to float64
    <= 2x the CPU fp32 gradient's + 1e-5 (here the fp32 noise is the only difference)."""
    import mvs_oracle
    from cameras import camera_batch, depth_range
    from conftest import record_parity
    from weights import deterministic_state_dict
    from mvs_amd import warp_and_assemble_cost_volume
    from mvs_amd.config import MVSConfig
    from mvs_amd.model import MVSNet
    B, V, D, H, W = 2, 3, 16, 256, 320
    h, w = H // 4, W // 4
    net = MVSNet(MVSConfig(d_num=D, in_h=H, in_w=W), device=torch.device("cpu"))
    net.load_state_dict(deterministic_state_dict(net.state_dict(), seed=99))
    net.train()
    net_c, net_d = copy.deepcopy(net), copy.deepcopy(net).double()
    net_g = copy.deepcopy(net).to(DEV)
    rng = np.random.default_rng(78)
    img = torch.from_numpy(rng.standard_normal((B * V, 3, H, W), dtype=np.float32))
    K, R, T = camera_batch(B, V, h, w)
    d_min, d_int = depth_range(B, d_int=4.0, distinct=True)
    wr = torch.from_numpy(rng.standard_normal((B, 1, D, h, w), dtype=np.float32))

    feats = net_g.feature_encoder(img.to(DEV))
    cv, _, _ = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, feats, B, V, d_num=D)
    (net_g.cost_volume_reg(cv) * wr.to(DEV)).sum().backward()

    feats = net_c.feature_encoder(img)
    wp, _, _ = mvs_oracle.homography_warping(K, R, T, d_min, d_int, feats, B, V, D, concat_growth=False)
    (net_c.cost_volume_reg.forward_full(mvs_oracle.assemble_cost_volume(wp, V)) * wr).sum().backward()

    feats = net_d.feature_encoder(img.double())
    cv64 = mvs_oracle.cost_volume_torch64(feats, K, R, T, d_min, d_int, B, V, D)
    (net_d.cost_volume_reg.forward_full(cv64) * wr.double()).sum().backward()

    pg, pc, pd = (dict(n.named_parameters()) for n in (net_g, net_c, net_d))
    # depthmap_refine is not on this loss's path (no gradient on any side)
    assert all((pg[n].grad is None) == (pd[n].grad is None) for n in pd)
    errs = {n: (_rel(pg[n].grad.cpu(), pd[n].grad), _rel(pc[n].grad, pd[n].grad)) for n in sorted(pd)
            if pd[n].grad is not None}
    record_parity("train_mode_smooth_loss_grads", grad_rel_l2_gpu_vs_f64_max=max(v[0] for v in errs.values()),
                  grad_rel_l2_cpu_vs_f64_max=max(v[1] for v in errs.values()),
                  per_parameter={k: [float(a), float(b)] for k, (a, b) in errs.items()})
    for name, (e_g, e_c) in errs.items():
        assert e_g <= 2.0 * e_c + 1e-5, "%s: GPU grad %.3g from float64, CPU fp32 %.3g" % (name, e_g, e_c)
    assert any(k.startswith("feature_encoder") for k in errs)
