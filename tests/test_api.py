"""CPU: the reference-facing API (names, signatures, state_dict layout, quirks) and that the
product path refuses to run without the HIP device (no CPU fallback)."""
import inspect
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN


def test_reference_signatures():
    from mvs_amd import homography_warping, assemble_cost_volume, extract_depth_map
    from mvs_amd.model import MVSNet
    assert list(inspect.signature(homography_warping).parameters)[:9] == [
        "K_batch", "R_batch", "T_batch", "d_min", "d_int", "feature_maps", "batch_size", "n_views",
        "d_num"]
    assert list(inspect.signature(assemble_cost_volume).parameters) == ["warped_feature_maps", "n_views"]
    assert list(inspect.signature(extract_depth_map).parameters)[:2] == ["prob_volume", "d_batch"]
    assert list(inspect.signature(MVSNet.forward).parameters) == [
        "self", "nn_input", "K_batch", "R_batch", "T_batch", "d_min", "d_int", "batch_size", "n_views"]


def test_state_dict_matches_reference():
    from mvs_amd.model import MVSNet
    ref = json.load(open(os.path.join(GOLDEN, "state_dict_keys.json")))
    net = MVSNet(device=torch.device("cpu"))
    ours = [[k, list(v.shape)] for k, v in net.state_dict().items()]
    assert ours == ref["keys"]                                  # same order, names and shapes
    assert sum(p.numel() for p in net.parameters) == ref["n_params"] == 382016
    assert isinstance(net.parameters, list)                     # model.py:164-166 quirk kept


def test_config_constants():
    from mvs_amd import config
    assert (config.D_SCALE, config.D_NUM, int(config.N_DEPTH_EST)) == (25, 20, 5)
    assert (config.FEAT_H, config.FEAT_W) == (128, 160)
    assert config.PAD == (11, 65, 81) and config.OUTPAD == (1, 1, 1)
    c = config.MVSConfig(d_num=192)
    assert c.pad == (97, 65, 81) and c.outpad == (1, 1, 1)


def test_depth_hypotheses_and_indices_match_reference():
    import mvs_oracle
    from mvs_amd.homography import depth_hypotheses, reference_indices
    d_min = torch.tensor([425.0, 500.0]).reshape(2, 1, 1, 1)
    d_int = torch.tensor([2.5, 1.0]).reshape(2, 1, 1, 1)
    assert torch.equal(depth_hypotheses(d_min, d_int, 7), mvs_oracle.depth_planes(d_min, d_int, 7))
    ref0, _, _ = mvs_oracle.view_indices(4, 3)
    assert torch.equal(reference_indices(4, 3), ref0)


def test_no_cpu_fallback():
    from mvs_amd import _lib, warp_and_assemble_cost_volume, extract_depth_map, assemble_cost_volume
    feat = torch.zeros(3, 4, 8, 8)
    K = torch.eye(3).repeat(3, 1, 1)
    with pytest.raises(_lib.MVSLibraryError):
        warp_and_assemble_cost_volume(K, K, torch.zeros(3, 3, 1), torch.ones(1, 1, 1, 1),
                                      torch.ones(1, 1, 1, 1), feat, 1, 3, d_num=4)
    with pytest.raises(_lib.MVSLibraryError):
        extract_depth_map(torch.rand(1, 1, 6, 4, 4), torch.arange(6.0).reshape(1, 6, 1, 1))
    with pytest.raises(_lib.MVSLibraryError):
        assemble_cost_volume(torch.zeros(3, 4, 5, 6, 7), 3)


def test_fake_kernels_give_shapes():
    """torch.library fake kernels (meta shapes) for graph capture / compile."""
    from torch._subclasses.fake_tensor import FakeTensorMode
    from mvs_amd import ops
    with FakeTensorMode():
        feat = torch.empty(6, 32, 16, 20)
        K = torch.empty(6, 3, 3)
        cv, ws = ops.cost_volume(feat, K, K, torch.empty(6, 3, 1), torch.empty(2), torch.empty(2),
                                 2, 3, 0, 12, 25.0)
        assert tuple(cv.shape) == (2, 32, 12, 16, 20) and ws.shape[0] >= 6 * 12 * 9
        w = ops.homography_warp(feat, K, K, torch.empty(6, 3, 1), torch.empty(2), torch.empty(2),
                                2, 3, 0, 12, 25.0)
        assert tuple(w.shape) == (6, 32, 12, 16, 20)
        d = ops.extract_depth_map_op(torch.empty(2, 1, 12, 16, 20), torch.empty(2, 12), 5)
        assert tuple(d.shape) == (2, 1, 16, 20)


def test_fake_kernels_refuse_in_place_side_outputs():
    """The ops that raise bound words / write batch sums in place (undeclared mutations) are eager-only:
    their fake kernels -- what torch.compile / functionalization trace -- raise when such an output is
    passed, and give shapes without one."""
    from torch._subclasses.fake_tensor import FakeTensorMode
    from mvs_amd import ops
    with FakeTensorMode():
        x = torch.empty(1, 5, 6, 7, 16)
        w = torch.empty(27, 16, 16)
        y = ops.conv3d_region_split(x, None, w, ops.CONV_S1, [5, 6, 7], [0, 0, 0], [5, 6, 7], [0, 0, 0],
                                    [5, 6, 7], None, torch.empty(ops.BOUND_WORDS, dtype=torch.int32), None, None)
        assert tuple(y.shape) == (1, 5, 6, 7, 16)
        with pytest.raises(NotImplementedError, match="eager mode only"):
            ops.conv3d_region_split(x, None, w, ops.CONV_S1, [5, 6, 7], [0, 0, 0], [5, 6, 7], [0, 0, 0],
                                    [5, 6, 7], None, torch.empty(ops.BOUND_WORDS, dtype=torch.int32), None,
                                    torch.empty(ops.BOUND_WORDS, dtype=torch.int32))
        with pytest.raises(NotImplementedError, match="eager mode only"):
            ops.conv2d(torch.empty(1, 8, 16, 16), torch.empty(8, 8, 3, 3), 1,
                       y_bound=torch.empty(ops.BOUND_WORDS, dtype=torch.int32))


def test_shard_helpers():
    from mvs_amd.depth_shards import plane_shard, owned_samples
    assert [plane_shard(256, 8, r) for r in (0, 7)] == [(0, 32), (224, 32)]
    with pytest.raises(ValueError):
        plane_shard(250, 8, 0)
    assert owned_samples(5, 2, 0) == [0, 2, 4] and owned_samples(1, 8, 3) == []


def test_derived_parameter_cache_follows_parameter_state():
    """ops.derived: a cached kernel-layout weight / eval-BN scale is reformed after any in-place
    update of its inputs (optimizer step, load_state_dict, running statistics) and never cached
    while autograd records."""
    import torch
    from mvs_amd.ops import derived
    w = torch.randn(4, 3)
    calls = []

    def f(t):
        calls.append(1)
        return t * 2.0

    with torch.no_grad():
        a = derived("t", (w,), f)
        b = derived("t", (w,), f)
        assert b is a and len(calls) == 1
        w.add_(1.0)   # in-place: version bump -> recomputed
        c = derived("t", (w,), f)
        assert len(calls) == 2 and torch.equal(c, w * 2.0)
    p = torch.nn.Parameter(torch.randn(3))
    derived("t", (p,), f)
    derived("t", (p,), f)
    assert len(calls) == 4   # requires_grad under grad mode: never cached


def test_derived_cache_keeps_one_entry_per_tensor_and_device():
    """ops.derived holds only the latest state per (tag, tensors): version bumps replace the entry
    (no growth over optimizer steps), a different target device is a different state, and the entry
    is evicted with its tensor."""
    import gc
    import torch
    from mvs_amd import ops
    w = torch.randn(5)
    calls = []

    def f(t):
        calls.append(1)
        return t + 1.0

    with torch.no_grad():
        n0 = len(ops._DERIVED)
        for _ in range(50):
            w.mul_(1.0)
            ops.derived("dev", (w,), f, "cuda:0")
        assert len(ops._DERIVED) == n0 + 1 and len(calls) == 50
        ops.derived("dev", (w,), f, "cuda:0")
        assert len(calls) == 50
        ops.derived("dev", (w,), f, "cuda:1")          # another target device: recomputed
        ops.derived("dev", (w,), f, "cuda:0")          # and back
        assert len(calls) == 52 and len(ops._DERIVED) == n0 + 1
        del w
        gc.collect()
        assert len(ops._DERIVED) == n0                  # evicted with its tensor
        ops.clear_derived()
        assert not ops._DERIVED


def test_select_images_matches_indexing():
    """model._select_images: a strided view for the reference indices 0, V, 2V, ... (no host sync on
    the GPU), plain indexing otherwise -- the same images either way."""
    import torch
    from mvs_amd.model import _select_images
    imgs = torch.randn(12, 3, 4, 5)
    for idx in (torch.tensor([0, 3, 6, 9]), torch.tensor([0]), torch.tensor([2, 5]), torch.tensor([1, 0, 4]),
                torch.tensor([0, 4, 8])):
        out = _select_images(imgs, idx)
        assert torch.equal(out, imgs[idx])
