"""Opt-in bf16 cost volume (reduced-precision cv behind a flag).

Parity bar: the bf16 kernel's output is BIT-IDENTICAL to the fp32 kernel's output rounded by torch's
own float -> bfloat16 conversion (round to nearest even), on the same inputs -- the variance is
computed in fp32 exactly as in the default path and rounded only in the store.  The fp32 path's
parity with the reference is covered in test_gpu_parity.py.  The backward passes the rounding
straight through: with the same (bf16-representable) upstream gradient it equals the fp32 op's
gradient up to the float-atomic summation order.
"""
import pytest
import torch

from cameras import camera_batch, depth_range, features

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.mark.parametrize("B,V,C,h,w,D", [(2, 3, 32, 128, 160, 48), (1, 2, 8, 24, 32, 7),
                                         (2, 5, 32, 64, 80, 16), (1, 3, 6, 9, 11, 5)])
def test_bf16_is_rounded_fp32(B, V, C, h, w, D):
    from mvs_amd import warp_and_assemble_cost_volume
    K, R, T = camera_batch(B, V, h, w)
    d_min, d_int = depth_range(B)
    f = features(B * V, C, h, w, seed=B * 100 + V).to(DEV)
    cv32, _, _ = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, f, B, V, d_num=D)
    cv16, _, _ = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, f, B, V, d_num=D,
                                               cv_dtype=torch.bfloat16)
    assert cv16.dtype == torch.bfloat16 and cv16.shape == cv32.shape
    assert torch.equal(cv16.view(torch.int16), cv32.to(torch.bfloat16).view(torch.int16))


def test_bf16_depth_shard_and_single_view():
    from mvs_amd import warp_and_assemble_cost_volume
    B, V, C, h, w, D = 1, 3, 8, 32, 40, 12
    K, R, T = camera_batch(B, V, h, w)
    d_min, d_int = depth_range(B)
    f = features(B * V, C, h, w, seed=9).to(DEV)
    full, _, _ = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, f, B, V, d_num=D,
                                               cv_dtype=torch.bfloat16)
    shard, _, _ = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, f, B, V, d_num=D, d_begin=5,
                                                d_count=4, cv_dtype=torch.bfloat16)
    assert torch.equal(shard.view(torch.int16), full[:, :, 5:9].view(torch.int16))
    one, _, _ = warp_and_assemble_cost_volume(K[:1], R[:1], T[:1], d_min, d_int, f[:1], 1, 1,
                                              d_num=D, cv_dtype=torch.bfloat16)
    assert torch.count_nonzero(one.float()) == 0


def test_bf16_backward_is_straight_through():
    from mvs_amd import ops
    B, V, C, h, w, D = 1, 3, 8, 24, 32, 6
    K, R, T = camera_batch(B, V, h, w)
    d_min, d_int = depth_range(B)
    f = features(B * V, C, h, w, seed=4).to(DEV)
    g = torch.randn(B, C, D, h, w, generator=torch.Generator().manual_seed(2)).to(torch.bfloat16)
    grads = []
    for op in (ops.cost_volume, ops.cost_volume_bf16):
        x = f.clone().requires_grad_(True)
        cv, _ = op(x, K, R, T, d_min, d_int, B, V, 0, D, 25.0)
        (cv.float() * g.to(DEV).float()).sum().backward()
        grads.append(x.grad.detach().cpu())
    scale = grads[0].abs().max().item()
    assert (grads[0] - grads[1]).abs().max().item() <= 1e-5 * max(scale, 1.0)


@pytest.mark.timeout(400)   # first bf16 Conv3d use compiles MIOpen kernels on a fresh box (~2 min)
def test_bf16_mvsnet_runs_close_to_fp32():
    """End to end with the opt-in: bf16 cv + bf16-autocast regulariser.  No parity claim against
    the reference (reduced precision by design); bounded against the fp32 model: median relative
    depth difference < 1 %."""
    from weights import deterministic_state_dict
    from mvs_amd.config import MVSConfig
    from mvs_amd.model import MVSNet
    B, V, D, H, W = 1, 3, 24, 256, 320
    K, R, T = camera_batch(B, V, H // 4, W // 4)
    d_min, d_int = depth_range(B)
    img = torch.randn(B * V, 3, H, W, generator=torch.Generator().manual_seed(5)).to(DEV)
    outs = []
    for dt in ("float32", "bfloat16"):
        net = MVSNet(MVSConfig(d_num=D, in_h=H, in_w=W, cv_dtype=dt))
        net.load_state_dict(deterministic_state_dict(net.state_dict()))
        net = net.to(DEV).eval()
        with torch.no_grad():
            outs.append([o.float().cpu() for o in net(img, K, R, T, d_min, d_int, B, V)])
    for a, b in zip(outs[0], outs[1]):
        assert torch.isfinite(b).all()
        rel = ((a - b).abs() / a.abs().clamp_min(1.0)).median().item()
        assert rel < 1e-2, rel
