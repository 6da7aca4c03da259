"""Train-mode BatchNorm parameters in one launch (ops.bn_train_params, csrc/channel_ops.hip; test.py:61's
model.train() under no_grad) against the device-op formulation it replaces (model._bn_train,
model._border_class_sums, model._bn_constant): the parameters, the running statistics and
num_batches_tracked after the update."""
import copy
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

DEV = torch.device("cuda", 0)


@pytest.mark.gpu
@pytest.mark.parametrize("border", [False, True])
def test_bn_train_params_matches_device_ops(border):
    from mvs_amd import model as M
    from mvs_amd.ops import bn_train_params
    g = torch.Generator().manual_seed(3 + int(border))
    C, Cp, n, bsz = 32, 32, (24, 20, 26), 2
    count = float(bsz * n[0] * n[1] * n[2])
    bn = torch.nn.BatchNorm3d(C, momentum=0.1).to(DEV)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-1, 1)
        bn.running_var.uniform_(0.5, 2)
    vals = torch.randn(int(count) // 8, C, generator=g, dtype=torch.float64) * 0.7 + 0.3
    s1 = (vals.sum(0) * 8).to(DEV)
    s2 = ((vals * vals).sum(0) * 8).to(DEV)
    ref = copy.deepcopy(bn)
    args = None
    if border:
        reg = M._grow(M._tconv_input_region(tuple((0, d - 1) for d in n), n, [13, 11, 14]), n, 1)
        weight = (torch.randn(C, Cp, 3, 3, 3, generator=g) * 0.1).to(DEV)
        prev = torch.stack((torch.rand(Cp, generator=g) + 0.5, torch.randn(Cp, generator=g) * 0.2,
                            torch.randn(Cp, generator=g) * 0.2)).to(DEV)
        c1, c2 = M._border_class_sums(weight, M._bn_constant(tuple(prev)), reg, n, bsz)
        want = M._bn_train(ref, s1 + c1, s2 + c2, count)
        args = M._border_tables_u(weight, reg, n, bsz) + (prev,)
    else:
        want = M._bn_train(ref, s1, s2, count)
    with torch.no_grad():
        got = bn_train_params(bn, s1, s2, count, args)
    for k in range(3):
        torch.testing.assert_close(got[k], want[k].detach().float(), rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(bn.running_mean, ref.running_mean, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(bn.running_var, ref.running_var, rtol=1e-6, atol=1e-7)
    assert bn.num_batches_tracked.item() == ref.num_batches_tracked.item() == 1
