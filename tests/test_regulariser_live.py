"""CPU: the eval-mode live-region regulariser (CostVolumeReg.forward_live) against the full-volume
op sequence of the reference (model.py:100-126, CostVolumeReg.forward_full).

Both evaluate the same sums of the same products for every output element (forward_live skips only
structurally-zero products of the n//2+1 padding and outputs no later layer reads); they differ by
fp32 summation order only.  Shapes cover even/odd/degenerate extents of D, H and W."""
import pytest
import torch

from mvs_amd.config import pad_outpad
from mvs_amd.model import CostVolumeReg


def _reg(D, h, w, seed=0):
    torch.manual_seed(seed)
    pad, outpad = pad_outpad(D, h, w)
    m = CostVolumeReg(pad=pad, outpad=outpad)
    for mod in m.modules():   # non-trivial eval statistics: BN(0) != 0 outside the live regions
        if isinstance(mod, torch.nn.BatchNorm3d):
            mod.running_mean.uniform_(-0.5, 0.5)
            mod.running_var.uniform_(0.5, 2.0)
            mod.weight.data.uniform_(0.5, 1.5)
            mod.bias.data.uniform_(-0.5, 0.5)
    return m


@pytest.mark.parametrize("shape", [(8, 12, 16), (7, 9, 11), (20, 32, 40), (5, 6, 6), (2, 3, 4),
                                   (1, 2, 3), (3, 1, 5), (48, 32, 40), (13, 10, 17)])
def test_live_region_equals_full_volume(shape):
    D, h, w = shape
    m = _reg(D, h, w).eval()
    cv = torch.rand(2, 32, D, h, w, generator=torch.Generator().manual_seed(D * 1000 + h))
    with torch.no_grad():
        full = m.forward_full(cv)
        live = m(cv)
    assert live.shape == full.shape == (2, 1, D, h, w)
    torch.testing.assert_close(live, full, rtol=1e-5, atol=1e-7)


def _bn_state(m):
    return {k: v.clone() for k, v in m.state_dict().items() if "BN_" in k}


@pytest.mark.parametrize("shape", [(8, 12, 16), (7, 9, 11), (20, 32, 40), (5, 6, 6), (2, 3, 4),
                                   (1, 2, 3), (3, 1, 5), (13, 10, 17)])
def test_train_mode_bn_live_equals_full_volume(shape):
    """Train-mode BN (test.py:61: model.train() under no_grad) normalises with batch statistics of
    the whole volume.  forward_live_train forms them from the live regions plus the structurally
    constant parts (zeros of conv_k_0, the 27 border classes of conv_k_1 of a constant field) and
    must give forward_full's probabilities AND running statistics (each BN updated once per use,
    in the reference's order)."""
    D, h, w = shape
    m1 = _reg(D, h, w, seed=3).train()
    m2 = _reg(D, h, w, seed=3).train()
    cv = torch.rand(2, 32, D, h, w, generator=torch.Generator().manual_seed(7 * D + w))
    with torch.no_grad():
        assert m1.live_train_ok(cv.shape[2:])
        live = m1(cv)
        full = m2.forward_full(cv)
    assert live.shape == full.shape == (2, 1, D, h, w)
    torch.testing.assert_close(live, full, rtol=1e-4, atol=1e-6)
    s1, s2 = _bn_state(m1), _bn_state(m2)
    for k in s2:
        torch.testing.assert_close(s1[k], s2[k], rtol=1e-5, atol=1e-6, msg=k)


def test_train_mode_bn_with_grad_uses_full_volume():
    """Autograd in train mode (train.py) keeps the reference op sequence (forward_full)."""
    m = _reg(8, 12, 16).train()
    cv = torch.rand(1, 32, 8, 12, 16, requires_grad=True)
    assert not m.live_train_ok(cv.shape[2:]) or not torch.is_grad_enabled()
    a = m(cv)
    m2 = _reg(8, 12, 16).train()
    b = m2.forward_full(cv)
    assert torch.equal(a, b)


@pytest.mark.parametrize("taps", [False, True])
@pytest.mark.parametrize("shape", [(8, 12, 16), (7, 9, 11), (5, 6, 6), (2, 3, 4), (3, 1, 5), (13, 10, 17)])
def test_train_mode_live_autograd_equals_full_volume(shape, taps, monkeypatch):
    """train.py:97-104 (model.train(), loss.backward()) through forward_live_train: the same function
    of the volume and the parameters as forward_full, so in float64 the outputs, the gradients w.r.t.
    the volume, every conv weight and every BN affine parameter, and the running statistics agree to
    rounding (CostVolumeReg.live_autograd_ok routes HIP fp32 training through it).  ``taps``: the
    region convolutions through the HIP path's per-tap GEMM boxes (tap_gemm.conv3d_box /
    conv_transpose3d_box), here in float64 on the CPU."""
    if taps:
        from mvs_amd import model as model_mod
        monkeypatch.setattr(model_mod, "_taps", lambda x: torch.is_grad_enabled())
    D, h, w = shape
    ms = [_reg(D, h, w, seed=5).double().train() for _ in range(2)]
    cv = torch.rand(2, 32, D, h, w, generator=torch.Generator().manual_seed(D + 31 * w), dtype=torch.float64)
    g = torch.rand(2, 1, D, h, w, generator=torch.Generator().manual_seed(h), dtype=torch.float64)
    outs, xgrads = [], []
    for m, fn in zip(ms, (lambda m, x: m.forward_full(x), lambda m, x: m.forward_live_train(x))):
        x = cv.clone().requires_grad_(True)
        y = fn(m, x)
        (y * g).sum().backward()
        outs.append(y.detach())
        xgrads.append(x.grad)
    torch.testing.assert_close(outs[1], outs[0], rtol=1e-10, atol=1e-13)
    torch.testing.assert_close(xgrads[1], xgrads[0], rtol=1e-9, atol=1e-13)
    p_full, p_live = dict(ms[0].named_parameters()), dict(ms[1].named_parameters())
    for k, v in p_full.items():
        assert p_live[k].grad is not None, k
        scale = v.grad.abs().max().item() + 1e-30
        assert (p_live[k].grad - v.grad).abs().max().item() <= 1e-9 * scale, k
    s1, s2 = _bn_state(ms[1]), _bn_state(ms[0])
    for k in s2:
        torch.testing.assert_close(s1[k], s2[k], rtol=1e-10, atol=1e-12, msg=k)


def test_live_autograd_route_conditions():
    """live_autograd_ok: only on a HIP device in fp32 with grad enabled and train-mode BN (a CPU volume
    keeps forward_full, test_train_mode_bn_with_grad_uses_full_volume); MVS_TRAIN_LIVE=0 refuses."""
    m = _reg(8, 12, 16).train()
    cv = torch.rand(1, 32, 8, 12, 16)
    assert not m.live_autograd_ok(cv)


def test_live_region_disabled_flag():
    m = _reg(8, 12, 16).eval()
    m.live_region = False
    cv = torch.rand(1, 32, 8, 12, 16)
    with torch.no_grad():
        assert torch.equal(m(cv), m.forward_full(cv))


def test_live_region_gradients_match():
    """Autograd through forward_live (eval BN, e.g. fine-tuning with frozen statistics) gives the
    gradients of the full path w.r.t. the cost volume and the conv weights."""
    m = _reg(6, 8, 10).eval()
    cv = torch.rand(1, 32, 6, 8, 10)
    g = torch.rand(1, 1, 6, 8, 10)
    grads = []
    for fn in (m.forward_full, m.forward_live):
        x = cv.clone().requires_grad_(True)
        m.zero_grad()
        (fn(x) * g).sum().backward()
        grads.append((x.grad.clone(), m.conv_3_1.weight.grad.clone(), m.deconv_1_0.weight.grad.clone()))
    for a, b in zip(*grads):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-8)


def test_live_region_needs_matching_geometry():
    """A regulariser built for one geometry and run on another takes forward_full, which raises
    the reference's shape mismatch instead of returning wrongly indexed live regions."""
    m = _reg(8, 12, 16).eval()
    cv = torch.rand(1, 32, 10, 12, 16)
    assert not m._live_geometry_ok(cv.shape[2:])
    with torch.no_grad(), pytest.raises(RuntimeError):
        m(cv)
