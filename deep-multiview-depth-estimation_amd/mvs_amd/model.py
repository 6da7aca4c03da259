"""Drop-in ``MVSNet`` (reference ``scripts/model.py:155-207``) on the MI355X cost-volume path.

Module tree and ``state_dict`` keys are the reference's (93 entries: ``feature_encoder.model.N.*``,
``cost_volume_reg.{conv_*,deconv_*,BN_*}.*``, ``depthmap_refine.model.N.*``), so reference
checkpoints load unchanged, and ``forward`` has the reference signature:

    forward(nn_input, K_batch, R_batch, T_batch, d_min, d_int, batch_size, n_views)
        -> (initial_depth_map [B,1,h,w], refined_depth_map [B,1,h,w])

What changes is the hot path: ``model.py:177-181`` (per-plane kornia warp loop + torch.cat growth
+ 6-D variance) becomes ONE fused HIP kernel (``costvolume.warp_and_assemble_cost_volume``) and
``model.py:187`` the HIP soft-argmin.  The 2-D/3-D convolutions stay on PyTorch-ROCm (MIOpen),
as the north star prescribes.  Like the reference (``model.py:164-166``) the instance attribute
``parameters`` is a LIST of tensors (``train.py:160`` passes it to Adam); use
``named_parameters()`` / ``state_dict()`` for module-generic code.
"""
import warnings

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import config as cfg_mod
from .config import MVSConfig
from .costvolume import warp_and_assemble_cost_volume
from .depthmap import extract_depth_map

# (in, out, kernel, stride, padding) of the 2-D feature encoder (model.py:35-59), base_filt 8,
# DIM_REDUCE 4 -> 8 / 16 / 32 channels; BN+ReLU follow every conv but the last.
_ENCODER = [(3, 8, 3, 1, 1), (8, 8, 3, 1, 1), (8, 16, 5, 2, 2), (16, 16, 3, 1, 1),
            (16, 16, 3, 1, 1), (16, 32, 5, 2, 2), (32, 32, 3, 1, 1), (32, 32, 3, 1, 1)]
# refinement net (model.py:134-145): 4 -> 32 -> 32 -> 32 -> 1
_REFINE = [(4, 32, 3, 1, 1), (32, 32, 3, 1, 1), (32, 32, 3, 1, 1), (32, 1, 3, 1, 1)]


def _conv_bn_relu_stack(spec, device):
    layers = []
    for n, (cin, cout, k, s, p) in enumerate(spec):
        layers.append(nn.Conv2d(cin, cout, k, stride=s, padding=p, bias=False, device=device))
        if n + 1 < len(spec):
            layers += [nn.BatchNorm2d(cout, eps=1e-5, momentum=0.1, device=device), nn.ReLU()]
    return nn.Sequential(*layers)


class FeatureEncoder(nn.Module):
    """model.py:22-65 -- images [N,3,H,W] -> features [N,32,H/4,W/4]."""

    def __init__(self, in_ch=3, base_filt=8, device=None):
        super().__init__()
        if (in_ch, base_filt) != (3, 8):
            raise ValueError("the reference encoder is fixed at in_ch=3, base_filt=8")
        self.model = _conv_bn_relu_stack(_ENCODER, device)

    def forward(self, x):
        return self.model(x)


class CostVolumeReg(nn.Module):
    """model.py:68-126 -- 3-D regulariser + softmax over depth (dim 2).

    Four branches read the cost volume (conv_k_0, k = 0..3, 8/16/32/64 channels); the stride-2
    convs use padding dim//2+1 so every level stays at full resolution (config.py:20)."""

    def __init__(self, in_ch=32, base_filt=8, device=None, pad=None, outpad=None):
        super().__init__()
        pad = cfg_mod.PAD if pad is None else pad
        outpad = cfg_mod.OUTPAD if outpad is None else outpad
        f1, f2, f4, f8 = base_filt, 2 * base_filt, 4 * base_filt, 8 * base_filt
        c3 = lambda i, o, s, p: nn.Conv3d(i, o, 3, stride=s, padding=p, bias=False, device=device)
        d3 = lambda i, o: nn.ConvTranspose3d(i, o, 3, stride=2, padding=pad, output_padding=outpad,
                                             bias=False, device=device)
        self.conv_0_0 = c3(in_ch, f1, 1, 1)
        self.conv_1_0 = c3(in_ch, f2, 2, pad)
        self.conv_2_0 = c3(in_ch, f4, 2, pad)
        self.conv_3_0 = c3(in_ch, f8, 2, pad)
        self.conv_1_1 = c3(f2, f2, 1, 1)
        self.conv_2_1 = c3(f4, f4, 1, 1)
        self.conv_3_1 = c3(f8, f8, 1, 1)
        self.deconv_3_0 = d3(f8, f4)
        self.deconv_2_0 = d3(f4, f2)
        self.deconv_1_0 = d3(f2, f1)
        self.conv_out = c3(f1, 1, 1, 1)
        self.ReLU = nn.ReLU()
        self.BN_0 = nn.BatchNorm3d(f1, eps=1e-5, momentum=0.1, device=device)
        self.BN_1 = nn.BatchNorm3d(f2, eps=1e-5, momentum=0.1, device=device)
        self.BN_2 = nn.BatchNorm3d(f4, eps=1e-5, momentum=0.1, device=device)
        self.BN_3 = nn.BatchNorm3d(f8, eps=1e-5, momentum=0.1, device=device)
        self.Norm = nn.Softmax(2)

    def forward(self, cv):
        act = lambda bn, y: self.ReLU(bn(y))
        # the BN modules are shared between levels exactly as in model.py:101-121
        y0 = act(self.BN_0, self.conv_0_0(cv))
        y1 = act(self.BN_1, self.conv_1_0(cv))
        y2 = act(self.BN_2, self.conv_2_0(cv))
        y3 = act(self.BN_3, self.conv_3_0(cv))
        y1 = act(self.BN_1, self.conv_1_1(y1))
        y2 = act(self.BN_2, self.conv_2_1(y2))
        y3 = act(self.BN_3, self.conv_3_1(y3))
        y3 = act(self.BN_2, self.deconv_3_0(y3))
        y2 = act(self.BN_1, self.deconv_2_0(y3 + y2))
        y1 = act(self.BN_0, self.deconv_1_0(y2 + y1))
        return self.Norm(self.conv_out(y1 + y0))


class DepthRefinement(nn.Module):
    """model.py:129-152 -- residual refinement of the normalised depth."""

    def __init__(self, in_ch=4, base_filt=32, device=None):
        super().__init__()
        if (in_ch, base_filt) != (4, 32):
            raise ValueError("the reference refinement net is fixed at in_ch=4, base_filt=32")
        self.model = _conv_bn_relu_stack(_REFINE, device)

    def forward(self, depth_and_input):
        return self.model(depth_and_input) + depth_and_input[:, 0].unsqueeze(1)


class MVSNet(nn.Module):
    """model.py:155-207 with the fused MI355X cost volume.  ``cfg`` replaces the reference's
    import-time globals (D_NUM, D_SCALE, FEAT_H/W, PAD/OUTPAD); the default equals them."""

    def __init__(self, cfg: MVSConfig = None, device=None):
        super().__init__()
        self.cfg = cfg if cfg is not None else MVSConfig()
        self.feature_encoder = FeatureEncoder(device=device)
        self.cost_volume_reg = CostVolumeReg(device=device, pad=self.cfg.pad, outpad=self.cfg.outpad)
        self.depthmap_refine = DepthRefinement(device=device)
        # reference quirk kept for train.py:160 (Adam(model.parameters, ...)), model.py:164-166
        self.parameters = (list(self.feature_encoder.parameters()) +
                           list(self.cost_volume_reg.parameters()) +
                           list(self.depthmap_refine.parameters()))

    def forward(self, nn_input, K_batch, R_batch, T_batch, d_min, d_int, batch_size, n_views):
        c = self.cfg
        device = nn_input.device
        feature_maps = self.feature_encoder(nn_input)
        bf16 = c.cv_dtype == "bfloat16"
        cost_volume, d_batch, ref_views = warp_and_assemble_cost_volume(
            K_batch, R_batch, T_batch, d_min, d_int, feature_maps, batch_size, n_views,
            d_num=c.d_num, d_scale=c.d_scale,
            cv_dtype=torch.bfloat16 if bf16 else torch.float32)
        if bf16:   # opt-in: regulariser under bf16 autocast, fp32 probabilities
            with torch.autocast(device.type, dtype=torch.bfloat16):
                prob_volume = self.cost_volume_reg(cost_volume).float()
        else:
            prob_volume = self.cost_volume_reg(cost_volume)
        initial_depth_map = extract_depth_map(prob_volume, d_batch, c.n_depth_est)
        return initial_depth_map, self.refine(nn_input, initial_depth_map, d_min, d_int, ref_views)

    def refine(self, nn_input, initial_depth_map, d_min, d_int, ref_views):
        """model.py:189-205: normalise, concat the downsampled reference image, refine, rescale."""
        c = self.cfg
        device = initial_depth_map.device
        d_trans = d_min.to(device)
        d_span = d_int.to(device).mul(c.d_num).mul(c.d_scale)
        norm_depth = torch.div(torch.subtract(initial_depth_map, d_trans), d_span)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            ref_img = F.interpolate(nn_input[ref_views.to(nn_input.device)],
                                    (c.feat_h, c.feat_w), mode="bilinear")
        refined = self.depthmap_refine(torch.cat((norm_depth, ref_img), dim=1))
        return refined.mul(d_span).add(d_trans)
