"""Opt-in bf16 cost volume (reduced-precision cv behind a flag,
MVSConfig(cv_dtype="bfloat16")).

Parity bar: the bf16 kernels' output (NCDHW and channel-quad) is BIT-IDENTICAL to the fp32 kernel's
output rounded by torch's own float -> bfloat16 conversion (round to nearest even), on the same
inputs -- the variance is computed in fp32 exactly as in the default path and rounded only in the
store.  Downstream, the regulariser's HIP layers widen the bf16 quads to fp32 on load (exact), so the
whole bf16 inference step is BIT-IDENTICAL to the fp32 step run on the rounded volume.  The fp32
path's parity with the reference is covered in test_gpu_parity.py.  The backward passes the rounding
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


def test_bf16_mvsnet_runs_close_to_fp32():
    """End to end with the opt-in: bf16 cv, fp32 regulariser on the rounded values.  No parity
    claim against the reference (reduced precision by design); bounded against the fp32 model:
    median relative depth difference < 1 %."""
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


def _to_c4(x):
    b, c = x.shape[:2]
    return x.reshape((b, c // 4, 4) + tuple(x.shape[2:])).permute(0, 1, 3, 4, 5, 2).contiguous()


@pytest.mark.parametrize("B,V,C,h,w,D", [(2, 3, 32, 64, 80, 24), (1, 5, 8, 37, 53, 7), (1, 2, 4, 16, 16, 3)])
def test_bf16_channel_quad_is_rounded_fp32(B, V, C, h, w, D):
    """mvs::cost_volume_c4_bf16 == mvs::cost_volume_c4(...).to(bfloat16), bit for bit, also for a
    depth shard."""
    from mvs_amd import ops
    K, R, T = camera_batch(B, V, h, w)
    d_min, d_int = depth_range(B, d_int=6.0, distinct=True)
    f = features(B * V, C, h, w, seed=C + D).to(DEV)
    for d_begin, d_count in ((0, D), (D // 3, D - D // 3)):
        c32 = ops.cost_volume_c4(f, K, R, T, d_min, d_int, B, V, d_begin, d_count, 25.0)
        c16 = ops.cost_volume_c4_bf16(f, K, R, T, d_min, d_int, B, V, d_begin, d_count, 25.0)
        assert c16.dtype == torch.bfloat16 and c16.shape == c32.shape
        assert torch.equal(c16.view(torch.int16), c32.to(torch.bfloat16).view(torch.int16))


@pytest.mark.parametrize("cout,wino", [(8, True), (8, False), (1, False)])
def test_narrow_conv_reads_bf16_quads_exactly(cout, wino):
    """conv3d_k3 on the bf16 channel-quad volume == conv3d_k3 on the same values widened to fp32:
    the widening is exact and the arithmetic the fp32 kernel's (bit-equal)."""
    from mvs_amd.ops import conv3d_k3
    g = torch.Generator().manual_seed(cout)
    x = _to_c4(torch.randn(2, 32 if cout == 8 else 8, 9, 13, 37, generator=g)).to(torch.bfloat16).to(DEV)
    wt = (torch.randn(cout, x.shape[1] * 4, 3, 3, 3, generator=g) * 0.1).to(DEV)
    with torch.no_grad():
        a = conv3d_k3(x, wt, in_c4=True, wino_z=wino)
        b = conv3d_k3(x.float(), wt, in_c4=True, wino_z=wino)
    assert torch.equal(a, b)


@pytest.mark.parametrize("cout", [16, 32, 64])
def test_region_s2_reads_bf16_quads_exactly(cout):
    """conv3d_region (CONV_S2) on the bf16 channel-quad volume == on the widened fp32 quads."""
    from mvs_amd.config import pad_outpad
    from mvs_amd.model import _grow, _tconv_input_region
    from mvs_amd.ops import CONV_S2, conv3d_region, region_weight
    n = (24, 20, 26)
    pad, _ = pad_outpad(*n)
    Bx = _tconv_input_region(tuple((0, d - 1) for d in n), n, pad)
    out_reg = _grow(Bx, n, 1)
    g = torch.Generator().manual_seed(cout)
    x = _to_c4(torch.randn(2, 32, *n, generator=g)).to(torch.bfloat16).to(DEV)
    w27 = region_weight(torch.nn.Conv3d(32, cout, 3)).detach().to(DEV)
    args = (list(n), [lo for lo, _ in out_reg], [hi - lo + 1 for lo, hi in out_reg], None, None, list(pad))
    with torch.no_grad():
        a = conv3d_region(x, None, w27, CONV_S2, *args, in_c4=True)
        b = conv3d_region(x.float(), None, w27, CONV_S2, *args, in_c4=True)
    assert torch.equal(a, b)


@pytest.mark.parametrize("train_bn", [False, True])
def test_bf16_mvsnet_step_is_fp32_step_on_rounded_volume(train_bn):
    """MVSNet.forward with cv_dtype="bfloat16" (the HIP channel-quad bf16 feed; BN eval, and the
    test.py:61 train-mode-BN mode) == the fp32 network whose cost volume is rounded to bf16 and
    widened back, bit for bit (initial depth and BN running statistics)."""
    import copy
    from weights import deterministic_state_dict
    from mvs_amd import extract_depth_map, ops
    from mvs_amd.config import MVSConfig
    from mvs_amd.homography import depth_hypotheses
    from mvs_amd.model import MVSNet
    B, V, D, H, W = 2, 3, 16, 256, 320
    K, R, T = camera_batch(B, V, H // 4, W // 4)
    d_min, d_int = depth_range(B, d_int=4.0)
    img = torch.randn(B * V, 3, H, W, generator=torch.Generator().manual_seed(6)).to(DEV)
    net = MVSNet(MVSConfig(d_num=D, in_h=H, in_w=W, cv_dtype="bfloat16"))
    net.load_state_dict(deterministic_state_dict(net.state_dict()))
    net = net.to(DEV).train(train_bn)
    ref = copy.deepcopy(net)
    with torch.no_grad():
        ini, _ = net(img, K, R, T, d_min, d_int, B, V)
        feats = ref.feature_encoder(img)
        cv = ops.cost_volume_c4(feats, K, R, T, d_min, d_int, B, V, 0, D, 25.0)
        prob = ref.cost_volume_reg(cv.to(torch.bfloat16).float())
        d_batch = depth_hypotheses(d_min, d_int, D, 25).to(DEV)
        ini_ref = extract_depth_map(prob, d_batch)
    assert torch.equal(ini, ini_ref)
    if train_bn:
        sa, sb = net.cost_volume_reg.state_dict(), ref.cost_volume_reg.state_dict()
        for k in sb:
            assert torch.equal(sa[k], sb[k]), k
