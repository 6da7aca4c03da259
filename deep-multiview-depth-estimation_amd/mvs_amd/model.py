"""Drop-in ``MVSNet`` (reference ``scripts/model.py:155-207``) on the MI355X cost-volume path.

Module tree and ``state_dict`` keys are the reference's (93 entries: ``feature_encoder.model.N.*``,
``cost_volume_reg.{conv_*,deconv_*,BN_*}.*``, ``depthmap_refine.model.N.*``), so reference
checkpoints load unchanged, and ``forward`` has the reference signature:

    forward(nn_input, K_batch, R_batch, T_batch, d_min, d_int, batch_size, n_views)
        -> (initial_depth_map [B,1,h,w], refined_depth_map [B,1,h,w])

What changes is the hot path: ``model.py:177-181`` (per-plane kornia warp loop + torch.cat growth
+ 6-D variance) becomes ONE fused HIP kernel (``costvolume.warp_and_assemble_cost_volume``) and
``model.py:187`` the HIP soft-argmin.  In fp32 no-grad inference the 2-D encoder / refinement
convolutions and the 3-D regulariser's layers run on hand-written HIP kernels too (direct 2-D convs
with fused BN + ReLU, MFMA region convs on the live regions; conv_0_0 and
conv_1_0 on split-fp16 matrix-core kernels fed by the fused kernel's split volume, §3.5, exact-fp32
kernels with ``MVS_SPLIT_F16=0``).  Under autograd the regulariser's Conv3d / ConvTranspose3d run as
per-tap rocBLAS GEMMs with their own backward (``tap_gemm.py``) and the 2-D layers as
the PyTorch-ROCm modules; other dtypes and the full-volume reference leg (``forward_full`` without
grad) use PyTorch-ROCm (MIOpen).  Like
the reference (``model.py:164-166``) the instance attribute
``parameters`` is a LIST of tensors (``train.py:160`` passes it to Adam); use
``named_parameters()`` / ``state_dict()`` for module-generic code.
"""
import os
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


def _run_stack(seq, x, split_f16=False):
    """A conv -> BatchNorm -> ReLU stack (encoder / refinement).  In fp32 no-grad inference on the
    GPU the convolutions run on the direct HIP kernel (mvs::conv2d, csrc/conv2d_narrow.hip: exact fp32)
    with eval BN + ReLU fused into its epilogue; train-mode BN (test.py:61) takes one-pass float64
    batch sums of the convolution's output and one in-place BN + ReLU pass (csrc/channel_ops.hip),
    with the running statistics updated as torch does.  Elsewhere the modules themselves.
    ``split_f16`` (MVSConfig(arithmetic="split_f16"), opt-in): the 8..32-channel layers on the f16
    matrix cores with split operands (csrc/conv2d_split.hip)."""
    if _taps(x) and os.environ.get("MVS_TRAIN_CONV2D", "taps") == "taps":
        # under autograd on a HIP device (train.py:97-104): the convolutions as per-tap rocBLAS GEMMs
        # (tap_gemm.conv2d), not MIOpen's (its first training step compiles its kernels: ~40 s at cfg 2)
        from . import tap_gemm
        from .ops import conv2d_supported
        hip_fwd = os.environ.get("MVS_TRAIN_CONV2D_FWD", "hip") == "hip"
        for layer in seq:
            if isinstance(layer, nn.Conv2d) and hip_fwd and conv2d_supported(layer) and x.dim() == 4:
                x = tap_gemm.conv2d_hip_fwd(x, layer)   # the HIP forward kernel, per-tap-GEMM backward
            elif isinstance(layer, nn.Conv2d) and tap_gemm.conv2d_applies(layer):
                x = tap_gemm.conv2d(x, layer.weight, layer.stride, layer.padding)
            else:
                x = layer(x)
        return x
    if not _hip_inference(x):
        return seq(x)
    from .ops import (CONV2D_SPLIT_SHAPES, bn_relu_, bound_words, channel_stats, conv2d, conv2d_split,
                      conv2d_supported)
    layers = list(seq)
    # split-fp16 MFMA convolutions (csrc/conv2d_split.hip) for the 8..32-channel inputs: every layer's
    # output carries bound words (one zeroed set per layer, one memset) that scale the next layer's input
    words = (bound_words(len(layers), x.device)
             if split_f16 and os.environ.get("MVS_CONV2D_F16", "1") != "0" else None)

    def conv(layer, x, xb, yb, bn=None):
        """(y, whether yb now bounds y): the HIP convolutions for the reference's layer shapes"""
        if isinstance(layer, nn.Conv2d) and conv2d_supported(layer):
            k = layer.kernel_size[0]
            if xb is not None and (layer.in_channels, layer.out_channels, k, layer.stride[0]) in CONV2D_SPLIT_SHAPES:
                return conv2d_split(x, layer.weight, layer.stride[0], xb, yb, *(bn or ())), yb is not None
            return conv2d(x, layer.weight, layer.stride[0], *(bn or ()), y_bound=yb), yb is not None
        y = layer(x)
        if bn is None:
            return y, False
        return bn_relu_(y.contiguous(), False, *bn, y_bound=yb), yb is not None

    xb = None   # x's bound words (None: unknown)
    i = 0
    while i < len(layers):
        layer = layers[i]
        yb = None if words is None or not isinstance(layer, nn.Conv2d) else words[i]
        if (i + 2 < len(layers) and isinstance(layers[i + 1], nn.BatchNorm2d)
                and isinstance(layers[i + 2], nn.ReLU)):
            bn = layers[i + 1]
            if bn.running_mean is None or not bn.affine:   # no running statistics: the module
                return _run_tail(layers[i:], x)
            if bn.training:
                y = conv(layer, x, xb, None)[0].contiguous()
                x = bn_relu_(y, False, *_bn_train_hip(bn, *channel_stats(y, False), y.numel() // y.shape[1]),
                             y_bound=yb)
                bounded = yb is not None
            else:   # eval BN + ReLU fused into the convolution's epilogue
                x, bounded = conv(layer, x, xb, yb, _bn_eval(bn))
            i += 3
        else:
            x, bounded = conv(layer, x, xb, yb)
            i += 1
        xb = yb if bounded else None
    return x


def _bn_eval(bn):
    """Eval BatchNorm as (scale, shift, mean): y = (x - mean) * scale + shift, scale = weight /
    sqrt(running_var + eps) (torch's batch_norm_inference order); the scale is cached per parameter
    state (ops.derived)."""
    from .ops import derived
    eps = bn.eps
    scale = derived(("bn_scale", eps), (bn.weight, bn.running_var), lambda wt, var: wt / torch.sqrt(var + eps))
    return scale, bn.bias, bn.running_mean


def _run_tail(layers, x):
    for layer in layers:
        x = layer(x)
    return x


class FeatureEncoder(nn.Module):
    """model.py:22-65 -- images [N,3,H,W] -> features [N,32,H/4,W/4]."""

    def __init__(self, in_ch=3, base_filt=8, device=None):
        super().__init__()
        if (in_ch, base_filt) != (3, 8):
            raise ValueError("the reference encoder is fixed at in_ch=3, base_filt=8")
        self.model = _conv_bn_relu_stack(_ENCODER, device)
        self.split_f16 = False   # MVSNet.set_arithmetic

    def forward(self, x):
        return _run_stack(self.model, x, self.split_f16)


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
        self.pad, self.outpad = tuple(pad), tuple(outpad)
        # eval-mode live-region evaluation (see forward_live); False = always the full-volume path
        self.live_region = True
        # False (default, MVSConfig(arithmetic="fp32")): every HIP layer in exact fp32 (the depth-Winograd
        # VALU conv_0_0, fp32-MFMA region convs).  True (arithmetic="split_f16", opt-in, narrower than
        # fp32): the f16 matrix cores with split-fp16 operands (csrc/split.h) read the split cost volume
        self.split_f16 = False

    def forward(self, cv):
        """cv [B, C, D, H, W] (the reference's input), an ops.BoundCostVolume (the channel-quad layout
        [B, C/4, D, H, W, 4] fp32 or split int32 with its bound words, ops.cost_volume_c4_absmax /
        cost_volume_c4_split), the bf16 channel-quad volume of ops.cost_volume_c4_bf16 (opt-in), or a
        costvolume.DeferredCostVolume -- the volume's inputs, consumed where it is formed by the fused
        head kernel (forward_live_head) or materialised for any other path.  The HIP live paths read
        the channel-quad volumes in place; other paths get the reference layout in fp32."""
        from .costvolume import DeferredCostVolume
        from .ops import BoundCostVolume, unsplit_cost_volume
        if isinstance(cv, DeferredCostVolume):
            if self.head_ok(cv):
                return self.forward_live_head(cv)
            cv = cv.materialize()
        bound = None
        if isinstance(cv, BoundCostVolume):
            cv, bound = cv.data, cv.absmax
        elif cv.dim() == 6 and cv.dtype == torch.int32:
            raise ValueError("a split cost volume is meaningless without its bound words: pass "
                             "ops.BoundCostVolume(cv, absmax) (what warp_and_assemble_cost_volume returns)")
        if cv.dim() == 6:
            if self.live_ok(cv.shape[2:5]) and _hip_cv(cv):
                return self.forward_live(cv, bound)
            if (cv.dtype == torch.int32 and bound is not None and self.split_f16 and self.live_train_ok(cv.shape[2:5])
                    and _hip_cv(cv)):
                return self.forward_live_train(cv, bound)   # the split-fp16 train-mode path reads it as is
            if cv.dtype == torch.int32:   # the split cost volume: fp32 values back (to 2^-22) for other paths
                cv = unsplit_cost_volume(cv, bound)
            if self.live_train_ok(cv.shape[2:5]) and _hip_cv(cv):
                return self.forward_live_train(cv, bound)
            cv = cv.permute(0, 1, 5, 2, 3, 4).reshape((cv.shape[0], 4 * cv.shape[1]) + tuple(cv.shape[2:5])).float()
        if self.live_ok(cv.shape[2:]):
            return self.forward_live(cv)
        if self.live_train_ok(cv.shape[2:]):
            return self.forward_live_train(cv)
        if self.live_autograd_ok(cv):
            return self.forward_live_train(cv)   # (the torch layers: differentiable)
        return self.forward_full(cv)

    def live_autograd_ok(self, cv):
        """forward_live_train under autograd (train.py:97-104: model.train(), loss.backward()): the
        live-region evaluation is the same function of the volume and the parameters as forward_full
        (structural zeros and per-class constants are exact identities, not approximations), so its
        autograd gradient is forward_full's -- with the region layers on their live regions only (cfg 2:
        the stride-2 convs and the deeper levels on 1/8 .. 1/512 of the volume).  On a HIP device in fp32,
        train-mode BN with running statistics, the module's padding derived from the volume extent;
        MVS_TRAIN_LIVE=0 keeps forward_full."""
        bns = (self.BN_0, self.BN_1, self.BN_2, self.BN_3)
        return (self.live_region and torch.is_grad_enabled() and cv.is_cuda and cv.dtype == torch.float32
                and cv.dim() == 5 and not torch.is_autocast_enabled()
                and os.environ.get("MVS_TRAIN_LIVE", "1") != "0" and self._live_geometry_ok(tuple(cv.shape[2:]))
                and all(bn.training and bn.track_running_stats and bn.running_mean is not None and bn.affine
                        for bn in bns))

    def head_ok(self, dcv):
        """The fused head kernel applies to this deferred cost volume: eval-mode live regions with the
        split-fp16 convolutions, fp32 HIP inference, C = 32, 2-3 views, D even and every stride-2
        padding odd (the kernel's window ownership), MVS_CV_HEAD=1 (opt-in)."""
        n = tuple(dcv.shape[2:])
        return (os.environ.get("MVS_CV_HEAD", "0") == "1" and self.split_f16 and self.live_ok(n)
                and _hip_inference(dcv.feature_maps) and dcv.shape[1] == 32 and dcv.n_views in (2, 3)
                and n[0] % 2 == 0 and all(p % 2 == 1 for p in self.pad))

    def forward_live_head(self, dcv):
        """forward_live with the cost volume consumed where it is formed: one fused
        kernel (ops.cost_volume_head, csrc/cv_head.hip) forms the variance plane by plane on chip and
        applies conv_0_0 + BN_0 + ReLU (full volume) and conv_1_0 + BN_1 + ReLU (on halo(B)); the only
        part of the volume written is conv_2_0's input box (the stride-2 windows of halo(C2), which
        contain conv_3_0's), as the split cost volume.  The rest of the live evaluation is
        _forward_live_hip's."""
        n = tuple(dcv.shape[2:])
        full = tuple((0, d - 1) for d in n)
        B = _tconv_input_region(full, n, self.pad)
        C2 = _tconv_input_region(B, n, self.pad)
        C3 = _tconv_input_region(C2, n, self.pad)
        h1, h2 = _grow(B, n, 1), _grow(C2, n, 1)
        lo = [max(2 * a - p, 0) for (a, _), p in zip(h2, self.pad)]
        hi = [min(2 * b - p + 2, d - 1) + 1 for (_, b), p, d in zip(h2, self.pad, n)]
        y0, y1, box = dcv.head(self.conv_0_0.weight, _bn_eval(self.BN_0), self.conv_1_0.weight,
                               _bn_eval(self.BN_1), self.pad, [a for a, _ in h1], [b - a + 1 for a, b in h1],
                               lo, hi)
        return self._forward_live_hip(box.data, n, B, C2, C3, True, box.absmax, head=(y0, y1),
                                      cv_box=box.box_region())

    def live_train_ok(self, n):
        """forward_live_train applies: every BN in train mode with running statistics (test.py:61's
        `model.train()` under `torch.no_grad()`), no autograd, the module's padding derived from n."""
        bns = (self.BN_0, self.BN_1, self.BN_2, self.BN_3)
        return (self.live_region and not torch.is_grad_enabled() and self._live_geometry_ok(n)
                and all(bn.training and bn.track_running_stats and bn.running_mean is not None
                        and bn.affine for bn in bns))

    def live_ok(self, n):
        """forward_live applies (eval BN, live_region on, the module's padding derived from n)."""
        return self.live_region and not self._bn_uses_batch_stats() and self._live_geometry_ok(n)

    def _live_geometry_ok(self, n):
        """forward_live relies on every U-Net level having the cost volume's extent n, which holds
        when the module's padding is the one config.py:20-21 derives from n.  A module built for
        another D or resolution takes forward_full, which (like the reference) then fails with the
        shape mismatch at the level sums instead of returning wrongly indexed levels."""
        from .config import pad_outpad
        return (self.pad, self.outpad) == pad_outpad(*n)

    def _bn_uses_batch_stats(self):
        return any(bn.training or bn.running_mean is None
                   for bn in (self.BN_0, self.BN_1, self.BN_2, self.BN_3))

    def forward_live(self, cv, bound=None):
        """Eval-mode regulariser evaluated only where its values reach the output.

        The stride-2 convs pad every dim by n//2 + 1 (config.py:20), so output j of conv_k_0 reads
        inputs 2j-P .. 2j-P+2 and is exactly 0 outside the middle half of each dim; the stride-2
        transposed convs likewise only READ the middle half of their input (an input i lands on
        outputs 2i-P .. 2i-P+2, off the [0, n) output range elsewhere).  Tracing the U-Net back
        from the full-size output: deconv_1_0 needs its input on B (middle half), deconv_2_0 needs
        its input on C2 (the middle of B), deconv_3_0 on C3 -- so level k's convs are evaluated on
        its region only (+1 halo for the 3x3x3 stride-1 conv), with exact zero padding at the
        tensor's borders.  Every output element is the same sum of the same products as in
        forward_full (only structurally-zero products and discarded outputs are skipped); sums may
        be ordered differently by MIOpen's kernels for the smaller shapes (fp32 rounding level).
        Eval-mode BatchNorm is elementwise, so it commutes with the restriction; train-mode BN
        (batch statistics over the whole volume, test.py:61) uses forward_full.
        """
        act = lambda bn, y: self.ReLU(bn(y))
        c4 = cv.dim() == 6          # channel-quad cost volume (HIP path only, see forward)
        n = tuple(cv.shape[2:5])
        full = tuple((0, d - 1) for d in n)
        B = _tconv_input_region(full, n, self.pad)
        C2 = _tconv_input_region(B, n, self.pad)
        C3 = _tconv_input_region(C2, n, self.pad)
        if _hip_cv(cv):
            return self._forward_live_hip(cv, n, B, C2, C3, c4, bound)
        return self._forward_live_torch(cv, n, B, C2, C3)

    def forward_live_torch(self, cv):
        """forward_live through PyTorch's convolutions (MIOpen on a HIP device) whatever the mode:
        the same live regions, an implementation independent of the HIP kernels (test reference)."""
        n = tuple(cv.shape[2:5])
        full = tuple((0, d - 1) for d in n)
        B = _tconv_input_region(full, n, self.pad)
        C2 = _tconv_input_region(B, n, self.pad)
        C3 = _tconv_input_region(C2, n, self.pad)
        return self._forward_live_torch(cv, n, B, C2, C3)

    def _forward_live_torch(self, cv, n, B, C2, C3):
        act = lambda bn, y: self.ReLU(bn(y))
        full = tuple((0, d - 1) for d in n)
        # torch layers (CPU, autograd): the same regions through PyTorch's convolutions
        y0 = act(self.BN_0, self.conv_0_0(cv))
        # level 1 on B, level 2 on C2, level 3 on C3 (regions carry their origin in the volume)
        lv = []
        for conv_a, conv_b, bn, reg in ((self.conv_1_0, self.conv_1_1, self.BN_1, B),
                                        (self.conv_2_0, self.conv_2_1, self.BN_2, C2),
                                        (self.conv_3_0, self.conv_3_1, self.BN_3, C3)):
            halo = _grow(reg, n, 1)
            y = act(bn, _conv_s2_region(cv, conv_a.weight, halo, self.pad))
            lv.append(act(bn, _conv_s1_region(y, halo, conv_b.weight, reg, n)))
        y1, y2, y3 = lv
        y3 = act(self.BN_2, _tconv_region(y3, C3, self.deconv_3_0.weight, C2, self.pad))
        y2 = act(self.BN_1, _tconv_region(y3 + y2, C2, self.deconv_2_0.weight, B, self.pad))
        z = act(self.BN_0, _tconv_region(y2 + y1, B, self.deconv_1_0.weight, full, self.pad)) + y0
        return self.Norm(self.conv_out(z))

    def _forward_live_hip(self, cv, n, B, C2, C3, c4=False, bound=None, head=None, cv_box=(None, None)):
        """forward_live on the HIP kernels: conv_0_0 (csrc/conv3d_narrow.hip), every region conv
        and transposed conv on the fp32 MFMA with channels-last region tensors and the eval BN +
        ReLU fused (csrc/conv3d_region.hip), deconv_1_0 + BN_0 + ReLU + `+ y0` and the `y2 + y1`
        sum in one kernel (csrc/deconv3d_region.hip), conv_out (conv3d_narrow.hip).  ``c4``: cv is
        the channel-quad volume, read by conv_0_0 and the three stride-2 convs with 16-byte loads;
        ``bound``: its bound words (the split-fp16 kernels' scale).  ``head``: (y0, y1) from the fused
        head kernel (forward_live_head) -- conv_0_0's and conv_1_0's outputs; cv is then the split
        volume on conv_2_0's input box only, ``cv_box`` (origin, size) that box."""
        from .ops import (CONV_S1, CONV_S2, CONV_T2, bound_words, conv3d_k3, conv3d_k3_split, conv3d_region,
                          conv3d_region_split, conv_head_fp32, conv_s2_split, deconv3d_k3s2, region_weight,
                          softmax_depth, split_head, timed_kernel)
        org = lambda reg: [lo for lo, _ in reg]
        size = lambda reg: [hi - lo + 1 for lo, hi in reg]
        dims, pad = list(n), list(self.pad)

        bn_eval = _bn_eval

        # conv_0_0 (VALU-bound) runs on a side stream, concurrently with the region chain (MFMA /
        # memory-latency-bound) that does not need it until deconv_1_0.  (Round 3's fp32 kernels measured
        # no gain from levels 2-3 beside level 1: 6.21-6.25 against 6.18-6.22 ms per cfg-2 step,
        # profiles/r03e_reg_layers.log; the split-fp16 path below does gain: l1_side)
        main = torch.cuda.current_stream(cv.device)
        # the split cost volume (int32, csrc/split.h) always goes to the split-fp16 kernels; an fp32
        # channel-quad volume does when split_f16 is on and it carries bound words
        split_cv = c4 and cv.dtype == torch.int32
        bound = bound if split_cv or (c4 and self.split_f16 and cv.dtype == torch.float32) else None
        if split_cv and bound is None:
            raise ValueError("split cost volume without its bound words")
        # the split-fp16 conv_0_0 (MFMA, LDS-staged) gains nothing beside the region chain: both compete
        # for the same CUs (cfg 2: 5.67 ms serialised against 5.78 ms on a side stream,
        # profiles/r03/r03u_reg_layers.log); the exact-fp32 VALU kernel overlaps the MFMA chain
        side = main if bound is not None else _side_stream(cv.device)
        # the split-fp16 eval path also runs the stride-1 and transposed region convolutions on the f16
        # matrix cores (ops.conv3d_region_split, csrc/conv3d_region_split.hip; MVS_REGION_SPLIT=0: the
        # fp32-MFMA kernels): every region tensor they read carries bound words, raised by the kernel
        # that writes it -- rows 0-2 conv_k_0's outputs, 3-5 conv_k_1's, 6 deconv_3_0's (one memset)
        bw = bound_words(7, cv.device) if split_cv and os.environ.get("MVS_REGION_SPLIT", "1") != "0" else None
        y1_bounded = False
        if head is None and split_cv and self._split_head_ok(cv, n):
            # conv_0_0 + BN_0 + ReLU and conv_1_0 + BN_1 + ReLU in one pass over the split volume
            # (ops.split_head, csrc/cv_head.hip PRESPLIT mode): bit-equal to the two kernels below
            h1 = _grow(B, n, 1)
            head = split_head(cv, bound, self.conv_0_0.weight, *bn_eval(self.BN_0), self.conv_1_0.weight,
                              *bn_eval(self.BN_1), pad, org(h1), size(h1), None if bw is None else bw[0])
            y1_bounded = bw is not None
        # the exact-fp32 head (ops.conv_head_fp32, csrc/conv3d_narrow.hip C1), opt-in (MVS_FP32_HEAD=1):
        # conv_1_0 on the fp32 matrix cores inside conv_0_0's VALU kernel, from the same LDS tiles, then
        # conv_1_1 behind it on the side stream.  Measured slower: the fused kernel 3.60 ms against
        # 1.88 + 1.15 ms for the two kernels alone, the cfg-2 step 6.6-6.7 against 5.8 ms (packed or single
        # fp32 FMAs, padded channel planes: 3.61-4.10 ms; gpurun_out r6i / r6j) -- the f32 MFMA does not
        # co-issue beside the packed-f32 VALU stream, it takes the same SIMD cycles
        y1_done = None
        if head is None and bound is None and self._fp32_head_ok(cv, c4, pad):
            h1 = _grow(B, n, 1)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                y0, y1a = conv_head_fp32(cv, self.conv_0_0.weight, *bn_eval(self.BN_0), self.conv_1_0.weight,
                                         *bn_eval(self.BN_1), pad, org(h1), size(h1))
                y1_done = conv3d_region(y1a, None, region_weight(self.conv_1_1), CONV_S1, dims, org(B), size(B),
                                        org(h1), size(h1), None, *bn_eval(self.BN_1), out_ncdhw=True)
            cv.record_stream(side)
        elif head is not None:
            y0, y1_head = head
        else:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                if bound is not None:
                    y0 = conv3d_k3_split(cv, bound, self.conv_0_0.weight, *bn_eval(self.BN_0))
                    bound.record_stream(side)
                else:
                    with timed_kernel("conv_0_0"):   # (bench.py's roofline kernel in fp32 arithmetic)
                        y0 = conv3d_k3(cv, self.conv_0_0.weight, *bn_eval(self.BN_0), in_c4=c4, wino_z=True)
            cv.record_stream(side)

        def level(k, conv_a, conv_b, bn, reg):
            halo = _grow(reg, n, 1)
            ab = None if bw is None else bw[k]   # ya's bound words
            if head is not None and reg is B:
                ya = y1_head   # conv_1_0 + BN_1 + ReLU on halo(B), from the head kernel
                ab = ab if y1_bounded else None
            elif bound is not None and conv_a.weight.shape[0] == 16:
                # conv_1_0 reads the whole volume: LDS-staged split-fp16 kernel (csrc/conv3d_s2_split.hip)
                ya = conv_s2_split(cv, bound, conv_a.weight, dims, org(halo), size(halo), pad, *bn_eval(bn))
                ab = None
            elif split_cv and bw is not None:
                # conv_2_0 / conv_3_0 on the split-fp16 matrix cores, straight from the split volume
                ya = conv3d_region_split(cv, None, region_weight(conv_a), CONV_S2, dims, org(halo), size(halo),
                                         cv_box[0], cv_box[1], pad, bound, None, ab, *bn_eval(bn))
            else:
                ya = conv3d_region(cv, None, region_weight(conv_a), CONV_S2, dims, org(halo), size(halo), cv_box[0],
                                   cv_box[1], pad, *bn_eval(bn), in_c4=c4, absmax=bound if split_cv else None,
                                   y_bound=ab)
            # -> (output, channels-last?).  Level 1's output only feeds deconv_1_0's input sum: channels-first
            # for its loads on the fp32 path; the split path keeps it channels-last (deconv_2_0's epilogue
            # adds it, coalesced)
            if ab is not None:
                return conv3d_region_split(ya, None, region_weight(conv_b), CONV_S1, dims, org(reg), size(reg),
                                           org(halo), size(halo), None, ab, None, bw[3 + k], *bn_eval(bn),
                                           out_ncdhw=False), True
            return conv3d_region(ya, None, region_weight(conv_b), CONV_S1, dims, org(reg), size(reg),
                                 org(halo), size(halo), None, *bn_eval(bn), out_ncdhw=reg is B), reg is not B
        # (the fp32 path: the region chain on a high-priority stream, or levels 1 and 3 on side streams beside
        # level 2 as below, measured 5.99-6.93 against 5.86-5.89 ms per cfg-2 step -- not kept, gpurun_out r6g)
        l1_side = bw is not None and head is not None and os.environ.get("MVS_L1_SIDE", "1") != "0"
        if y1_done is not None:   # (level 1 ran behind the fp32 head on the side stream)
            y1, y1_cl = y1_done, False
        elif l1_side:
            # level 1's conv_1_1 (LDS-bound) on a side stream beside levels 2-3 (L2-bound per-lane convs):
            # cfg-2 eval step 3.89-4.00 -> 3.80-3.93 ms (same box, tools/gpu_r5_env_ab.sh r5l1)
            s1 = _side_stream(cv.device, 1)
            s1.wait_stream(main)
            with torch.cuda.stream(s1):
                y1, y1_cl = level(0, self.conv_1_0, self.conv_1_1, self.BN_1, B)
        else:
            y1, y1_cl = level(0, self.conv_1_0, self.conv_1_1, self.BN_1, B)
        l3_side = l1_side and os.environ.get("MVS_L3_SIDE", "1") != "0"
        if l3_side:   # level 3 on a second side stream beside level 2 (3.91-3.93 -> 3.84-3.88 ms, r5l3)
            s3 = _side_stream(cv.device, 2)
            s3.wait_stream(main)
            with torch.cuda.stream(s3):
                y3 = level(2, self.conv_3_0, self.conv_3_1, self.BN_3, C3)[0]
            y2 = level(1, self.conv_2_0, self.conv_2_1, self.BN_2, C2)[0]
            main.wait_stream(s3)
            y3.record_stream(main)
        else:
            y2 = level(1, self.conv_2_0, self.conv_2_1, self.BN_2, C2)[0]
            y3 = level(2, self.conv_3_0, self.conv_3_1, self.BN_3, C3)[0]
        if l1_side:
            main.wait_stream(s1)
            y1.record_stream(main)
        if bw is not None:
            # deconv_3_0 + BN_2 + ReLU, then `+ y2` (model.py:119) in its epilogue: deconv_2_0 reads one tensor
            y32 = conv3d_region_split(y3, None, region_weight(self.deconv_3_0), CONV_T2, dims, org(C2), size(C2),
                                      org(C3), size(C3), pad, bw[5], None, bw[6], *bn_eval(self.BN_2), y_addend=y2)
            # and, when level 1 ran split (channels-last), deconv_2_0's epilogue forms model.py:121's y2 + y1:
            # deconv_1_0 reads one channels-last tensor (else deconv_1_0 adds the channels-first y1 on load)
            y2 = conv3d_region_split(y32, None, region_weight(self.deconv_2_0), CONV_T2, dims, org(B), size(B),
                                     org(C2), size(C2), pad, bw[6], None, None, *bn_eval(self.BN_1),
                                     out_ncdhw=not y1_cl, y_addend=y1 if y1_cl else None)
            if y1_cl:
                y1 = None
        else:
            y3 = conv3d_region(y3, None, region_weight(self.deconv_3_0), CONV_T2, dims, org(C2), size(C2),
                               org(C3), size(C3), pad, *bn_eval(self.BN_2))
            y2 = conv3d_region(y3, y2, region_weight(self.deconv_2_0), CONV_T2, dims, org(B), size(B), org(C2),
                               size(C2), pad, *bn_eval(self.BN_1), out_ncdhw=True)
        if side != main:   # (a stream waiting on itself is an event + barrier packet: a 6 us bubble)
            main.wait_stream(side)
            y0.record_stream(main)
            if y1_done is not None:
                y1.record_stream(main)
        z = deconv3d_k3s2(y2, org(B), self.deconv_1_0.weight, dims, pad, *bn_eval(self.BN_0), y0, x2=y1,
                          channels_last=bw is not None and y1_cl)
        return softmax_depth(conv3d_k3(z, self.conv_out.weight))

    def _fp32_head_ok(self, cv, c4, pad):
        """ops.conv_head_fp32 applies: the fp32 channel-quad volume of 32 channels, conv_1_0 32 -> 16,
        every stride-2 padding odd (the kernel's window ownership), MVS_FP32_HEAD=1 (opt-in: slower, above)."""
        return (os.environ.get("MVS_FP32_HEAD", "0") == "1" and c4 and cv.dtype == torch.float32
                and cv.dim() == 6 and cv.shape[1] == 8 and tuple(self.conv_1_0.weight.shape[:2]) == (16, 32)
                and all(p % 2 == 1 for p in pad))

    def _split_head_ok(self, cv, n):
        """ops.split_head applies to this split volume: C = 32 (8 channel quads), D even and every
        stride-2 padding odd (the kernel's window ownership), MVS_SPLIT_HEAD not 0."""
        return (os.environ.get("MVS_SPLIT_HEAD", "1") != "0" and cv.shape[1] == 8 and n[0] % 2 == 0
                and all(p % 2 == 1 for p in self.pad))

    def forward_live_train(self, cv, bound=None):
        """Train-mode-BatchNorm regulariser (test.py:53,61: `model.train()` under `no_grad`)
        evaluated on live regions, exactly.

        With batch statistics every BN normalises by the mean / variance over the WHOLE volume, so
        the full-size tensors matter through their sums -- but most of them are structurally
        constant (the eval-mode argument of forward_live, carried through BN):
          * conv_k_0 (stride 2, padding n//2+1) is exactly 0 outside its middle-half region M, so
            its BN statistics are the region's sums over the full element count, and
            relu(BN(conv_k_0)) is the per-channel constant a_k = relu(BN(0)) outside M;
          * conv_k_1 (3x3x3, padding 1) of that field is, outside M grown by 1 (R1), a constant per
            channel and volume-border class (which of its taps fall inside the volume): 27 classes
            with known voxel counts, so its statistics are the R1 region's sums plus
            count x value (and count x value^2) per class;
          * the stride-2 transposed convs read only the middle half M of their input (forward_live),
            so deconv_3_0 / deconv_2_0 / deconv_1_0 are computed from the M-region tensors; their
            statistics need the full output, computed here in full (it is not constant).
        Every BatchNorm updates its running statistics once per use, in the reference's order
        (BN_0, BN_1, BN_2, BN_3, BN_1, BN_2, BN_3, BN_2, BN_1, BN_0), as forward_full does."""
        act = lambda y, bn: self.ReLU(_apply_bn(y, *bn))
        n = tuple(cv.shape[2:5])
        full = tuple((0, d - 1) for d in n)
        M = _tconv_input_region(full, n, self.pad)
        R1, R2 = _grow(M, n, 1), _grow(M, n, 2)
        bsz = cv.shape[0]
        count = bsz * n[0] * n[1] * n[2]
        if _hip_cv(cv):
            return self._forward_live_train_hip(cv, n, full, M, R1, R2, count, bound)
        y0 = _narrow_conv(self.conv_0_0, cv)
        y0 = act(y0, _bn_train(self.BN_0, *_sums(y0), count))
        stage = []
        convs_a = ((self.conv_1_0, self.BN_1), (self.conv_2_0, self.BN_2), (self.conv_3_0, self.BN_3))
        # the three stride-2 convs read the same volume over the same region R2: ONE convolution with their
        # output channels stacked (under autograd one input layout pass, one input gradient)
        zs = _conv_s2_region(cv, torch.cat([c.weight for c, _ in convs_a], 0), R2, self.pad,
                             splits=tuple(c.weight.shape[0] for c, _ in convs_a))   # 0 outside M
        zs = zs.split([c.weight.shape[0] for c, _ in convs_a], 1)
        for z, (conv_a, bn) in zip(zs, convs_a):
            p = _bn_train(bn, *_sums(z), count)
            stage.append((act(z, p), _bn_constant(p)))              # relu(BN(0)) outside M
        lv = []
        for (y, a), conv_b, bn in zip(stage, (self.conv_1_1, self.conv_2_1, self.conv_3_1),
                                      (self.BN_1, self.BN_2, self.BN_3)):
            z = _conv_s1_region(y, R2, conv_b.weight, R1, n)
            s1, s2 = _sums(z)
            c1, c2 = _border_class_sums(conv_b.weight, a, R1, n, bsz)
            p = _bn_train(bn, s1 + c1, s2 + c2, count)
            lv.append(_crop_pad(act(z, p), R1, M, n))
        y1, y2, y3 = lv
        # (the full outputs for the statistics; BN + ReLU on M only, the next layer's input)
        z = _tconv_region(y3, M, self.deconv_3_0.weight, full, self.pad, n)
        y3 = act(_crop_pad(z, full, M, n), _bn_train(self.BN_2, *_sums(z), count))
        z = _tconv_region(y3 + y2, M, self.deconv_2_0.weight, full, self.pad, n)
        y2 = act(_crop_pad(z, full, M, n), _bn_train(self.BN_1, *_sums(z), count))
        z = _tconv_region(y2 + y1, M, self.deconv_1_0.weight, full, self.pad)
        z = act(z, _bn_train(self.BN_0, *_sums(z), count)) + y0
        return self.Norm(_narrow_conv(self.conv_out, z))

    def _forward_live_train_hip(self, cv, n, full, M, R1, R2, count, bound=None):
        """forward_live_train on the HIP kernels: raw (BN-free) region convs on the fp32 MFMA
        (conv3d_region.hip), conv_0_0 / conv_out (conv3d_narrow.hip), deconv_1_0
        (deconv3d_region.hip); batch statistics as float64 sums of the raw outputs; BN + ReLU
        applied in place to the region tensors (channels-last).  The transposed convs run over
        the full output volume (their statistics) and keep the M-region part.  ``cv`` may be the
        channel-quad volume (conv_0_0 and the stride-2 convs read it with 16-byte loads)."""
        from .ops import (CONV_S1, CONV_S2, CONV_T2, bn_relu_, bound_words, channel_stats, conv3d_k3,
                          conv3d_k3_split, conv3d_region, conv3d_region_split_sums, conv_s2_split_multi_sums,
                          deconv3d_k3s2, region_weight, softmax_depth)
        c4 = cv.dim() == 6
        # with split_f16 the stride-1 and transposed convs run on the split-fp16 matrix cores
        # (conv3d_region_split): their inputs' bound words are raised by the BN + ReLU passes -- rows 0-2
        # the conv_k_1 inputs, 4-5 conv_2_1 / conv_3_1's outputs, 6 deconv_3_0's (raw when the transposed
        # convs fold the BN + ReLU into their staging: `fold`)
        bw = (bound_words(7, cv.device) if self.split_f16 and os.environ.get("MVS_REGION_SPLIT", "1") != "0"
              else None)
        bwr = lambda k: None if bw is None else bw[k]
        org = lambda reg: [lo for lo, _ in reg]
        size = lambda reg: [hi - lo + 1 for lo, hi in reg]
        dims, pad, bsz = list(n), list(self.pad), cv.shape[0]
        # conv_0_0 and its batch statistics on a side stream, concurrently with the region chain
        main = torch.cuda.current_stream(cv.device)
        side = _side_stream(cv.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            if bound is not None and c4 and self.split_f16 and cv.shape[1] == 8:
                # (fp32 channel quads with their bound words, or the split volume itself)
                # the channel-quad volume with its bound words: conv_0_0 on the split-fp16 matrix cores
                # (fp32-level error; 4.4 -> ~1 ms at cfg 2), raw output for the batch sums
                y0 = conv3d_k3_split(cv, bound, self.conv_0_0.weight)
            else:
                y0 = conv3d_k3(cv, self.conv_0_0.weight, in_c4=c4, wino_z=True)
            p0 = _bn_train_hip(self.BN_0, *channel_stats(y0, False), count)
        cv.record_stream(side)
        stage = []
        zs = None
        if cv.dtype == torch.int32 and os.environ.get("MVS_S2_MULTI", "1") != "0":
            # conv_1_0, conv_2_0, conv_3_0 read the same split volume over the same region R2: one launch
            # (ops.conv_s2_split_multi_sums), the volume's operands loaded once for all three
            zs = conv_s2_split_multi_sums(cv, [region_weight(c) for c in (self.conv_1_0, self.conv_2_0,
                                                                          self.conv_3_0)],
                                          dims, org(R2), size(R2), pad, bound, y_bound=bwr(0))
        for k, (conv_a, bn) in enumerate(((self.conv_1_0, self.BN_1), (self.conv_2_0, self.BN_2),
                                          (self.conv_3_0, self.BN_3))):
            if zs is not None:
                z, s1, s2 = zs[k]
            elif cv.dtype == torch.int32:   # the split volume: conv_k_0 on the split-fp16 matrix cores, the
                # batch sums formed in its epilogue
                z, s1, s2 = conv3d_region_split_sums(cv, None, region_weight(conv_a), CONV_S2, dims, org(R2),
                                                     size(R2), None, None, pad, bound)
            else:
                z = conv3d_region(cv, None, region_weight(conv_a), CONV_S2, dims, org(R2), size(R2), None, None,
                                  pad, in_c4=c4)
                s1, s2 = channel_stats(z, True)
            p = _bn_train_hip(bn, s1, s2, count)
            if zs is not None and bw is not None and k < 2:
                # conv_1_1 / conv_2_1's LDS kernels apply relu(BN(.)) in their staging: z stays raw, its
                # bound the three outputs' (row 0)
                stage.append(((z, p), p))
            else:
                stage.append((bn_relu_(z, True, *p, y_bound=bwr(k if zs is None or bw is None else 2)), p))
            # (p: relu(BN(0)) outside M)
        lv = []
        # conv_2_1 / conv_3_1's BN + ReLU (and deconv_3_0's, with the + y2 sum) applied in the transposed
        # convs' LDS staging instead of a pass over each tensor (ops.conv3d_region_split_sums x_bn / x2_bn)
        fold = bw is not None and os.environ.get("MVS_T2_FOLD", "1") != "0"
        def level_b(k, y, pa, conv_b, bn):
            # level 1 only feeds deconv_1_0's input sum: channels-first for its loads
            cf = bn is self.BN_1
            if bw is not None:   # sums over R1 in the epilogue, only M stored (the next layers read M)
                if isinstance(y, tuple):   # (raw conv_k_0 output, its BN): folded into the staging
                    xin, xbn, xbw = y[0], y[1], bw[0]
                else:
                    xin, xbn, xbw = y, None, bw[k if zs is None else 2]
                z, s1, s2 = conv3d_region_split_sums(xin, None, region_weight(conv_b), CONV_S1, dims, org(R1),
                                                     size(R1), org(R2), size(R2), None, xbw, out_ncdhw=cf,
                                                     store_origin=org(M), store_size=size(M),
                                                     y_bound=bw[3 + k] if fold and not cf else None, x_bn=xbn)
            else:
                z = conv3d_region(y, None, region_weight(conv_b), CONV_S1, dims, org(R1), size(R1), org(R2),
                                  size(R2), None, out_ncdhw=cf)
                s1, s2 = channel_stats(z, not cf)
                z = (_crop_cf if cf else _crop_cl)(z, R1, M)
            p = _bn_train_hip(bn, s1, s2, count, border=(conv_b.weight, R1, n, bsz, pa))
            if fold and not cf:
                return (z, p)   # raw, with its BN: normalised in the transposed conv's staging
            return bn_relu_(z, not cf, *p, y_bound=None if cf else bwr(3 + k))

        # conv_1_1 and conv_2_1 on two side streams beside conv_3_1 (independent until the transposed convs;
        # each BN's running-statistic updates stay in order: the stream waits for main before and main for
        # it after): train-mode step 11.9 -> 11.7 ms (same box, tools/gpu_r5_env_ab.sh r5tls)
        lstreams = (bw is not None and os.environ.get("MVS_TRAIN_LEVEL_STREAMS", "1") != "0")
        args = list(zip(stage, (self.conv_1_1, self.conv_2_1, self.conv_3_1), (self.BN_1, self.BN_2, self.BN_3)))
        lv = [None, None, None]
        used = []
        for k in (0, 1, 2):
            (y, pa), conv_b, bn = args[k]
            if lstreams and k < 2:
                st = _side_stream(cv.device, 1 + k)
                st.wait_stream(main)
                with torch.cuda.stream(st):
                    lv[k] = level_b(k, y, pa, conv_b, bn)
                used.append((st, lv[k]))
            else:
                lv[k] = level_b(k, y, pa, conv_b, bn)
        for st, out in used:
            main.wait_stream(st)
            for t in (out if isinstance(out, tuple) else (out,)):
                t.record_stream(main)
        y1, y2, y3 = lv
        if fold:
            (z3, p3), (z2, p2) = y3, y2
            z, s1, s2 = conv3d_region_split_sums(z3, None, region_weight(self.deconv_3_0), CONV_T2, dims, [0, 0, 0],
                                                 dims, org(M), size(M), pad, bw[5], y_bound=bw[6],
                                                 store_origin=org(M), store_size=size(M), x_bn=p3)
            p = _bn_train_hip(self.BN_2, s1, s2, count)
            # deconv_2_0 reads relu(BN_2(deconv_3_0)) + relu(BN_2(conv_2_1)) (model.py:119-120), both formed
            # in its staging from the raw tensors
            z, s1, s2 = conv3d_region_split_sums(z, z2, region_weight(self.deconv_2_0), CONV_T2, dims, [0, 0, 0],
                                                 dims, org(M), size(M), pad, bw[6], x2_bound=bw[4], out_ncdhw=True,
                                                 store_origin=org(M), store_size=size(M), x_bn=p, x2_bn=p2)
            p = _bn_train_hip(self.BN_1, s1, s2, count)
            c1 = y1.shape[1]
            one, zero = torch.ones(c1, device=y1.device), torch.zeros(c1, device=y1.device)
            y2 = bn_relu_(z, False, *p, r=y1, r_bn=(one, zero, zero))
            y1 = z3 = z2 = None
        elif bw is not None:
            # the transposed convs over the full output (their batch sums, formed in the epilogue), only
            # M stored: the next layer reads M
            z, s1, s2 = conv3d_region_split_sums(y3, None, region_weight(self.deconv_3_0), CONV_T2, dims,
                                                 [0, 0, 0], dims, org(M), size(M), pad, bw[5],
                                                 store_origin=org(M), store_size=size(M))
            p = _bn_train_hip(self.BN_2, s1, s2, count)
            # relu(BN_2(deconv_3_0)) + y2 (model.py:119) formed in the BN pass: y2 >= 0 (a ReLU output), so
            # relu((y2 - 0) * 1 + 0) is y2 exactly; deconv_2_0 then reads one tensor
            c2 = y2.shape[-1]
            one, zero = torch.ones(c2, device=y2.device), torch.zeros(c2, device=y2.device)
            y3 = bn_relu_(z, True, *p, r=y2, r_bn=(one, zero, zero), y_bound=bw[6])
            z, s1, s2 = conv3d_region_split_sums(y3, None, region_weight(self.deconv_2_0), CONV_T2, dims,
                                                 [0, 0, 0], dims, org(M), size(M), pad, bw[6], out_ncdhw=True,
                                                 store_origin=org(M), store_size=size(M))
            p = _bn_train_hip(self.BN_1, s1, s2, count)
            # relu(BN_1(deconv_2_0)) + y1 (model.py:121) formed in the BN pass (y1 >= 0: exact, as above)
            c1 = y1.shape[1]
            one, zero = torch.ones(c1, device=y1.device), torch.zeros(c1, device=y1.device)
            y2 = bn_relu_(z, False, *p, r=y1, r_bn=(one, zero, zero))
            y1 = None
        else:
            z = conv3d_region(y3, None, region_weight(self.deconv_3_0), CONV_T2, dims, [0, 0, 0], dims, org(M),
                              size(M), pad)
            p = _bn_train_hip(self.BN_2, *channel_stats(z, True), count)
            y3 = bn_relu_(_crop_cl(z, full, M), True, *p)
            del z
            z = conv3d_region(y3, y2, region_weight(self.deconv_2_0), CONV_T2, dims, [0, 0, 0], dims, org(M),
                              size(M), pad, out_ncdhw=True)
            p = _bn_train_hip(self.BN_1, *channel_stats(z, False), count)
            y2 = bn_relu_(_crop_cf(z, full, M), False, *p)
        del z
        z = deconv3d_k3s2(y2, org(M), self.deconv_1_0.weight, dims, pad, None, None, None, None, x2=y1)
        main.wait_stream(side)
        for t in (y0,) + tuple(p0):
            t.record_stream(main)
        p = _bn_train_hip(self.BN_0, *channel_stats(z, False), count)
        if os.environ.get("MVS_OUT_FOLD", "1") != "0":
            # relu(BN_0(deconv_1_0)) + relu(BN_0'(conv_0_0)) formed in conv_out's staging (one pass over the
            # full volume fewer)
            return softmax_depth(conv3d_k3(z, self.conv_out.weight, x2=y0, in_bn=torch.cat((p, p0))))
        z = bn_relu_(z, False, *p, r=y0, r_bn=p0)   # relu(BN_0(deconv_1_0)) + relu(BN_0'(conv_0_0))
        return softmax_depth(conv3d_k3(z, self.conv_out.weight))

    def forward_full(self, cv):
        act = lambda bn, y: self.ReLU(bn(y))
        # the BN modules are shared between levels exactly as in model.py:101-121; the two narrow
        # full-resolution layers run on the HIP kernel in no-grad fp32 inference (_narrow_conv),
        # e.g. test.py:61's train-mode BatchNorm under no_grad; under autograd on a HIP device
        # (train.py:97-104) every convolution runs as per-tap rocBLAS GEMMs (tap_gemm.py: MIOpen's
        # backward solvers for these shapes take minutes per step)
        conv = _train_conv if cv.is_cuda and torch.is_grad_enabled() else (lambda m, x: m(x))
        y0 = act(self.BN_0, _narrow_conv(self.conv_0_0, cv))
        y1 = act(self.BN_1, conv(self.conv_1_0, cv))
        y2 = act(self.BN_2, conv(self.conv_2_0, cv))
        y3 = act(self.BN_3, conv(self.conv_3_0, cv))
        y1 = act(self.BN_1, conv(self.conv_1_1, y1))
        y2 = act(self.BN_2, conv(self.conv_2_1, y2))
        y3 = act(self.BN_3, conv(self.conv_3_1, y3))
        y3 = act(self.BN_2, conv(self.deconv_3_0, y3))
        y2 = act(self.BN_1, conv(self.deconv_2_0, y3 + y2))
        y1 = act(self.BN_0, conv(self.deconv_1_0, y2 + y1))
        return self.Norm(_narrow_conv(self.conv_out, y1 + y0))


_SIDE_STREAMS = {}
# the lane of MVSNet's sample-pipelined eval forward that is issuing kernels (0: none): every lane gets
# its own side streams, so two lanes' branches never serialise on one stream
_LANE = [0]


def _side_stream(device, which=0, priority=0):
    """Extra HIP streams per device (and pipeline lane) for independent branches of the inference step."""
    key = (torch.device(device).index, which, _LANE[0], priority)
    if key not in _SIDE_STREAMS:
        _SIDE_STREAMS[key] = torch.cuda.Stream(device, priority=priority)
    return _SIDE_STREAMS[key]


_UNIFORM = {}


def _uniform_depths(d_min, d_int):
    """Every sample has the same (d_min, d_int) -- DTU's 425 / 2.5 for every camera, and d_int = 1 in
    train.py:95 / test.py:84.  Only then is a chunk of samples' forward the whole batch's: image i uses
    the depth planes of sample i mod B (homography.py:24-26, view-major tiling), which changes with the
    chunk's B unless all rows are equal.  A device tensor's answer is cached per storage and version (one
    device-to-host read per new tensor)."""
    out = True
    for t in (d_min, d_int):
        if t.numel() <= 1:
            continue
        if t.device.type == "cpu":
            out = out and bool((t == t.reshape(-1)[0]).all())
            continue
        key = (t.data_ptr(), t._version, tuple(t.shape), str(t.device))
        hit = _UNIFORM.get(key)
        if hit is None:
            if len(_UNIFORM) > 256:
                _UNIFORM.clear()
            hit = _UNIFORM[key] = bool((t == t.reshape(-1)[0]).all().item())
        out = out and hit
    return out


def _lane_stream(device, lane):
    """The stream of pipeline lane ``lane`` (MVSNet._forward_pipelined)."""
    key = (torch.device(device).index, "lane", lane)
    if key not in _SIDE_STREAMS:
        _SIDE_STREAMS[key] = torch.cuda.Stream(device)
    return _SIDE_STREAMS[key]


def _hip_inference(x):
    """fp32 inference on a HIP device (no autograd, no autocast): the regulariser's hand-written
    full-resolution layers apply."""
    return (x.is_cuda and x.dtype == torch.float32 and not torch.is_grad_enabled()
            and not torch.is_autocast_enabled())


def _hip_cv(cv):
    """_hip_inference for the regulariser's input: also the bf16 channel-quad cost volume of the
    reduced-precision opt-in (its HIP layers widen it to fp32 on load) and the split cost volume
    (int32 elements of fp16 hi / lo parts, read by the split-fp16 kernels)."""
    return _hip_inference(cv) or (cv.is_cuda and cv.dim() == 6 and cv.dtype in (torch.bfloat16, torch.int32)
                                  and not torch.is_grad_enabled() and not torch.is_autocast_enabled())


def _narrow_conv(conv, x):
    """conv_0_0 (32 -> 8) / conv_out (8 -> 1) at full resolution: on a HIP device, in fp32 and
    without autograd, the hand-written kernel (mvs::conv3d_k3, csrc/conv3d_narrow.hip: MIOpen
    runs these narrow full-volume layers at a few TFLOP/s); under autograd on a HIP device the
    per-tap GEMMs (_train_conv); otherwise the module itself."""
    if _hip_inference(x):
        from .ops import conv3d_k3
        return conv3d_k3(x, conv.weight)
    if x.is_cuda and torch.is_grad_enabled():
        from . import narrow_train
        if narrow_train.applies(conv, x):   # HIP forward, input gradient and weight gradient
            return narrow_train.conv3d(conv, x)
        return _train_conv(conv, x)
    return conv(x)


def _train_conv(m, x):
    """A regulariser Conv3d / ConvTranspose3d under autograd on a HIP device: per-tap rocBLAS GEMMs
    with their own backward (tap_gemm.py) instead of MIOpen (fp32 in and out)."""
    from . import tap_gemm
    if x.dtype != torch.float32 or torch.is_autocast_enabled():
        return m(x)
    return tap_gemm.conv_module(m, x)


# ---- train-mode BatchNorm from sums (CostVolumeReg.forward_live_train) ----------------------
class _SumsFn(torch.autograd.Function):
    """(sum y, sum y^2) per channel in float64, with the backward as ONE fp32 pass
    g1 + 2 y g2 (autograd of the plain expression broadcasts the float64 gradients over the volume:
    float64 temporaries of twice its size, cfg 2 8 ms per 32-channel pass)."""

    @staticmethod
    def forward(ctx, y, cdim):
        red = [d for d in range(y.dim()) if d != cdim]
        ctx.save_for_backward(y)
        ctx.cdim = cdim
        return y.sum(red, dtype=torch.float64), (y * y).sum(red, dtype=torch.float64)

    @staticmethod
    def backward(ctx, g1, g2):
        (y,) = ctx.saved_tensors
        shape = [1] * y.dim()
        shape[ctx.cdim] = -1
        c = y.shape[ctx.cdim]
        g1 = (torch.zeros(c, dtype=y.dtype, device=y.device) if g1 is None else g1.to(y.dtype)).view(shape)
        g2 = (torch.zeros(c, dtype=y.dtype, device=y.device) if g2 is None else g2.to(y.dtype)).view(shape)
        return torch.addcmul(g1, y, 2.0 * g2), None


def _sums(y, cdim=1):
    """Per-channel sum and sum of squares of y (channels on dim cdim) in float64."""
    cdim = cdim % y.dim()
    if torch.is_grad_enabled() and y.requires_grad:
        return _SumsFn.apply(y, cdim)
    red = [d for d in range(y.dim()) if d != cdim]
    return y.sum(red, dtype=torch.float64), (y * y).sum(red, dtype=torch.float64)


def _bn_relu_(y, p, cdim):
    """In place: y = relu((y - mean) * scale + shift), channels on dim cdim (region tensors are
    channels-last: cdim = -1)."""
    scale, shift, mean = p
    shape = [1] * y.dim()
    shape[cdim] = -1
    v = lambda t: t.view(shape)
    return y.sub_(v(mean)).mul_(v(scale)).add_(v(shift)).clamp_min_(0.0)


def _crop_cf(x, x_reg, want):
    """The box `want` (inside x_reg) of a channels-first region tensor x [B, C, d, h, w], contiguous."""
    sl = [slice(lo - xlo, hi - xlo + 1) for (xlo, _), (lo, hi) in zip(x_reg, want)]
    return x[:, :, sl[0], sl[1], sl[2]].contiguous()


def _crop_cl(x, x_reg, want):
    """The box `want` (inside x_reg) of a channels-last region tensor x [B, d, h, w, C], contiguous."""
    sl = [slice(lo - xlo, hi - xlo + 1) for (xlo, _), (lo, hi) in zip(x_reg, want)]
    return x[:, sl[0], sl[1], sl[2], :].contiguous()


def _bn_train(bn, s1, s2, count):
    """Batch statistics of a train-mode BatchNorm from per-channel sums over `count` elements:
    returns (scale, shift, mean) with BN(x) = (x - mean) * scale + shift (biased variance), and
    updates bn's running statistics the way torch's batch_norm does (unbiased variance, momentum,
    num_batches_tracked)."""
    mean = s1 / count
    var = (s2 / count - mean * mean).clamp_min(0.0)
    with torch.no_grad():
        bn.num_batches_tracked.add_(1)
        m = bn.momentum if bn.momentum is not None else 1.0 / float(bn.num_batches_tracked)
        bn.running_mean.mul_(1.0 - m).add_(mean.to(bn.running_mean), alpha=m)
        bn.running_var.mul_(1.0 - m).add_((var * (count / max(count - 1, 1))).to(bn.running_var), alpha=m)
    scale = bn.weight / torch.sqrt(var.to(bn.weight.dtype) + bn.eps)
    return scale, bn.bias, mean.to(bn.weight.dtype)


def _apply_bn(y, scale, shift, mean):
    v = lambda t: t.view((1, -1) + (1,) * (y.dim() - 2))
    return (y - v(mean)) * v(scale) + v(shift)


def _bn_train_hip(bn, s1, s2, count, border=None):
    """_bn_train on the HIP path as ONE launch (ops.bn_train_params), returning the [3, C] parameters
    (scale, shift, mean); ``border``: None or (weight, region, n, batch, prev) -- conv_k_1's
    border-class term (_border_class_sums) with the previous BN's parameters ``prev``.  momentum=None
    (the cumulative average) takes the device-op path."""
    from .ops import bn_train_params
    if bn.momentum is None:
        if border is not None:
            weight, reg, n, bsz, prev = border
            c1, c2 = _border_class_sums(weight, _bn_constant(tuple(prev)), reg, n, bsz)
            s1, s2 = s1 + c1, s2 + c2
        return torch.stack([t.detach().float() for t in _bn_train(bn, s1, s2, count)])
    b = None
    if border is not None:
        weight, reg, n, bsz, prev = border
        b = _border_tables_u(weight, reg, n, bsz) + (prev,)
    return bn_train_params(bn, s1, s2, count, b)


def _border_tables_u(weight, reg, n, bsz):
    """(U [C_out, C_in, K], counts [K]) of _border_class_sums for the K border classes outside reg:
    U[o][i][k] = the sum of weight[o][i] over class k's in-volume taps (float64), counts = voxels of the
    class outside reg over the batch -- cached per weight state (ops.derived), so a forward only forms
    u = U a (mvs_bn_train_params)."""
    from .ops import derived

    def build(w):
        masks, cnt, inside = _border_class_tables(tuple(n), tuple(reg), w.device)
        u = torch.einsum("oiabc,xa,yb,zc->oixyz", w.detach().double(), masks[0], masks[1], masks[2])
        outer = lambda v: v[0].view(-1, 1, 1) * v[1].view(1, -1, 1) * v[2].view(1, 1, -1)
        count = bsz * (outer(cnt) - outer(inside))
        return u.reshape(u.shape[0], u.shape[1], -1).contiguous(), count.reshape(-1).contiguous()
    return derived(("border_u", tuple(reg), tuple(n), int(bsz)), (weight,), build, weight.device)


def _bn_constant(p):
    """relu(BN(0)) per channel: the value of a BN + ReLU output where its input is exactly 0."""
    scale, shift, mean = p
    return torch.relu(-mean * scale + shift)


def _border_classes(d, lo, hi):
    """One dim of size d under a 3-tap, stride-1, padding-1 conv: (taps inside the volume, voxels
    of the class, of them inside [lo, hi]) for the border / interior index classes."""
    spans = [(0, 0, (1,))] if d == 1 else (
        [(0, 0, (1, 2)), (d - 1, d - 1, (0, 1))] + ([(1, d - 2, (0, 1, 2))] if d > 2 else []))
    return [(taps, b - a + 1, max(0, min(b, hi) - max(a, lo) + 1)) for a, b, taps in spans]


_CLASS_TABLES = {}


def _border_class_tables(n, reg, device):
    """Per dim: (tap masks [classes, 3], class voxel counts, of them inside reg) as float64 device
    tensors, cached per (volume, region, device): formed once instead of by host-to-device copies in
    every train-mode forward (pageable copies stall the host's run-ahead)."""
    key = (n, reg, str(device))
    hit = _CLASS_TABLES.get(key)
    if hit is None:
        masks, cnt, inside = [], [], []
        for d, (lo, hi) in zip(n, reg):
            classes = _border_classes(d, lo, hi)
            masks.append(torch.tensor([[1.0 if k in taps else 0.0 for k in range(3)] for taps, _, _ in classes],
                                      dtype=torch.float64, device=device))
            cnt.append(torch.tensor([c for _, c, _ in classes], dtype=torch.float64, device=device))
            inside.append(torch.tensor([i for _, _, i in classes], dtype=torch.float64, device=device))
        if len(_CLASS_TABLES) > 64:
            _CLASS_TABLES.clear()
        hit = _CLASS_TABLES[key] = (masks, cnt, inside)
    return hit


def _border_class_sums(weight, a, reg, n, bsz):
    """Sums (value, value^2) per output channel of conv3d(field, weight, padding 1) over the
    voxels OUTSIDE reg, where the input field is the per-channel constant a everywhere the
    window of such a voxel reaches (in-volume taps only).  The output there depends only on the
    voxel's border class: sum_ci a[ci] * sum_(in-volume taps) weight[co, ci, tap].  All classes
    at once (a few device ops, no per-class launches)."""
    w = weight.double()
    masks, cnt, inside = _border_class_tables(tuple(n), tuple(reg), w.device)
    # the constant field's response summed over each class's in-volume taps
    wa = torch.einsum("oiabc,i->oabc", w, a.double())    # the field's response per tap
    u = torch.einsum("oabc,zc->oabz", wa, masks[2])
    u = torch.einsum("oabz,yb->oayz", u, masks[1])
    u = torch.einsum("oayz,xa->oxyz", u, masks[0])
    outer = lambda v: v[0].view(-1, 1, 1) * v[1].view(1, -1, 1) * v[2].view(1, 1, -1)
    count = bsz * (outer(cnt) - outer(inside))            # voxels of each class outside reg
    return (u * count).sum((1, 2, 3)), (u * u * count).sum((1, 2, 3))


# ---- live-region helpers (CostVolumeReg.forward_live).  A region is a tuple of inclusive
# (lo, hi) index ranges over (D, H, W); a region tensor holds the volume's values on it.
def _grow(reg, n, k):
    return tuple((max(lo - k, 0), min(hi + k, d - 1)) for (lo, hi), d in zip(reg, n))


def _tconv_input_region(out_reg, n, pad):
    """Inputs of a stride-2, kernel-3, padding-P transposed conv that reach outputs out_reg:
    input i lands on outputs 2i - P + t, t = 0..2."""
    return tuple((max(-((-(lo + p - 2)) // 2), 0), min((hi + p) // 2, d - 1))
                 for (lo, hi), d, p in zip(out_reg, n, pad))


def _crop_pad(x, x_reg, want, n):
    """Values of the region tensor x (on x_reg) over the index box `want` (may leave the volume:
    zeros there, i.e. the conv's zero padding).  `want` inside the volume must lie in x_reg."""
    sl, pads = [], []
    for (xlo, xhi), (lo, hi), d in zip(x_reg, want, n):
        a, b = max(lo, 0), min(hi, d - 1)
        assert xlo <= a and b <= xhi, "region tensor does not cover the requested box"
        sl.append(slice(a - xlo, b - xlo + 1))
        pads.append((a - lo, hi - b))
    y = x[:, :, sl[0], sl[1], sl[2]]
    flat = [v for pr in reversed(pads) for v in pr]   # F.pad order: W, H, D
    return F.pad(y, flat) if any(flat) else y


def _taps(x):
    """The live-region helpers' convolutions go through the per-tap GEMMs (tap_gemm: MIOpen's backward
    solvers for these shapes are naive): under autograd on a HIP device in fp32."""
    return x.is_cuda and torch.is_grad_enabled() and x.dtype == torch.float32 and not torch.is_autocast_enabled()


def _region_conv3d(x, weight, stride, padding):
    if _taps(x):
        from . import tap_gemm
        return tap_gemm.conv3d(x, weight, stride, padding)
    return F.conv3d(x, weight, stride=stride, padding=padding)


def _conv_s2_region(x, weight, out_reg, pad, splits=None):
    """conv3d(x, weight, stride 2, padding pad) on the output box out_reg (x: full volume).

    Output j reads inputs 2j - P .. 2j - P + 2.  The input box of out_reg usually leaves the volume
    by different amounts on the two sides (n even); instead of materialising an asymmetrically
    padded copy, the conv runs on the in-volume crop with a symmetric padding p >= both overhangs,
    p of the left overhang's parity (so the stride-2 grid stays aligned), and the wanted outputs
    are sliced out: every kept output reads exactly its own window."""
    n = tuple(x.shape[2:])
    if _taps(x):
        # the box itself as a dense tensor: output j - lo reads inputs 2 (j - lo) - pad_lo + t of the crop
        # starting at max(2 lo - P, 0) (tap_gemm.conv3d_box)
        from . import tap_gemm
        sl, pl = [], []
        for (lo, hi), p, d in zip(out_reg, pad, n):
            a, b = 2 * lo - p, 2 * hi - p + 2
            ca, cb = max(a, 0), min(b, d - 1)
            assert ca <= cb, "output box reads no input"
            sl.append(slice(ca, cb + 1))
            pl.append(ca - a)
        whole = all(s_.start == 0 and s_.stop == d for s_, d in zip(sl, n))
        from . import region_train
        if (whole and splits is not None and region_train.enabled(x, "s2") and x.shape[1] == 32
                and tuple(splits) in (region_train.S2_SPLITS, (16,), (32,), (64,))):
            return region_train.s2_box(x, weight, out_reg, pad, tuple(pl), tuple(splits))   # HIP forward
        if not whole:   # (a whole-extent slice: no copy back in the backward)
            x = x[:, :, sl[0], sl[1], sl[2]]
        return tap_gemm.conv3d_box(x, weight, 2, tuple(pl), tuple(hi - lo + 1 for lo, hi in out_reg))
    sl, pads, offs = [], [], []
    for (lo, hi), p, d in zip(out_reg, pad, n):
        a, b = 2 * lo - p, 2 * hi - p + 2
        ca, cb = max(a, 0), min(b, d - 1)
        assert ca <= cb, "output box reads no input"
        lp, rp = ca - a, b - cb
        ps = max(lp, rp)
        ps += (ps - lp) % 2
        sl.append(slice(ca, cb + 1))
        pads.append(ps)
        offs.append((ps - lp) // 2)
    y = _region_conv3d(x[:, :, sl[0], sl[1], sl[2]], weight, 2, tuple(pads))
    cnt = [hi - lo + 1 for lo, hi in out_reg]
    assert all(o + c <= m for o, c, m in zip(offs, cnt, y.shape[2:]))
    return y[:, :, offs[0]:offs[0] + cnt[0], offs[1]:offs[1] + cnt[1], offs[2]:offs[2] + cnt[2]]


def _conv_s1_region(x, x_reg, weight, out_reg, n):
    """conv3d(., weight, stride 1, padding 1) on out_reg, from the region tensor x on x_reg."""
    want = tuple((lo - 1, hi + 1) for lo, hi in out_reg)
    xin = _crop_pad(x, x_reg, want, n)
    from . import region_train
    if (_taps(x) and region_train.enabled(x, "s1") and weight.shape[0] == weight.shape[1]
            and weight.shape[0] in region_train.S1_CHANNELS):
        return region_train.s1_valid(xin, weight)   # HIP forward, per-tap-GEMM backward
    return _region_conv3d(xin, weight, 1, 0)


def _tconv_region(x, x_reg, weight, out_reg, pad, dims=None):
    """conv_transpose3d(., weight, stride 2, padding pad) on out_reg, from the region tensor x on
    x_reg (which must hold every input that reaches out_reg: _tconv_input_region)."""
    if _taps(x):
        # the box as a dense tensor (tap_gemm.conv_transpose3d_box: outputs past the inputs' reach are 0)
        from . import tap_gemm
        crop = []
        for (xlo, _), (lo, hi), p in zip(x_reg, out_reg, pad):
            assert lo - (2 * xlo - p) >= 0, "transposed-conv input region starts after the output box"
            crop.append(lo - (2 * xlo - p))
        from . import region_train
        if (dims is not None and region_train.enabled(x, "t2")
                and (weight.shape[0], weight.shape[1]) in region_train.T2_SHAPES):
            return region_train.t2_box(x, weight, x_reg, out_reg, pad, dims, tuple(crop))   # HIP forward
        return tap_gemm.conv_transpose3d_box(x, weight, 2, tuple(crop), tuple(hi - lo + 1 for lo, hi in out_reg))
    y = F.conv_transpose3d(x, weight, stride=2)   # output q <-> volume index 2 * xlo + q - P
    sl, pads = [], []
    for (xlo, _), (lo, hi), p, m in zip(x_reg, out_reg, pad, y.shape[2:]):
        o0 = 2 * xlo - p
        a, b = lo - o0, hi - o0
        assert a >= 0, "transposed-conv input region starts after the output box"
        sl.append(slice(a, min(b, m - 1) + 1))
        pads.append((0, max(b - (m - 1), 0)))   # outputs past the last input's reach are 0
    y = y[:, :, sl[0], sl[1], sl[2]]
    flat = [v for pr in reversed(pads) for v in pr]
    return F.pad(y, flat) if any(flat) else y


class DepthRefinement(nn.Module):
    """model.py:129-152 -- residual refinement of the normalised depth."""

    def __init__(self, in_ch=4, base_filt=32, device=None):
        super().__init__()
        if (in_ch, base_filt) != (4, 32):
            raise ValueError("the reference refinement net is fixed at in_ch=4, base_filt=32")
        self.model = _conv_bn_relu_stack(_REFINE, device)
        self.split_f16 = False   # MVSNet.set_arithmetic

    def forward(self, depth_and_input):
        return _run_stack(self.model, depth_and_input, self.split_f16) + depth_and_input[:, 0].unsqueeze(1)


def _select_images(images, idx):
    """images[idx] for the reference-view indices (homography.py:29-36 returns them as a CPU int64
    tensor 0, V, 2V, ...): a strided view when they form such a progression, since indexing a
    device tensor with a CPU index copies it to the device, and that pageable copy synchronises
    the host with every kernel queued before it (a bubble in each inference step)."""
    if idx.device.type == "cpu" and idx.dim() == 1 and idx.numel() > 0 and not idx.is_floating_point():
        n = idx.numel()
        first = int(idx[0])
        step = int(idx[1]) - first if n > 1 else 1
        if step > 0 and first >= 0 and torch.equal(idx, first + step * torch.arange(n, dtype=idx.dtype)) \
                and first + step * (n - 1) < images.shape[0]:
            return images[first:first + step * (n - 1) + 1:step]
    return images[idx.to(images.device)]


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
        self.set_arithmetic(self.cfg.arithmetic)
        # eval inference over B >= 2 samples: chunks of samples issued on their own streams (forward)
        # (measured slower at cfg 2: 6.32 against 5.87 ms per step with 2 chunks, gpurun_out r6f -- off)
        self.pipeline_chunks = int(os.environ.get("MVS_PIPELINE_CHUNKS", "1"))

    def set_arithmetic(self, arithmetic):
        """"fp32" (the reference's numerics: every HIP layer in exact fp32) or "split_f16" (opt-in: the
        encoder, refinement and regulariser convolutions on the f16 matrix cores with split-fp16
        operands, the cost volume stored as its fp16 hi / lo parts; narrower than fp32)."""
        from .config import ARITHMETICS
        if arithmetic not in ARITHMETICS:
            raise ValueError("arithmetic must be one of %s, got %r" % (ARITHMETICS, arithmetic))
        self.cfg.arithmetic = arithmetic
        split = arithmetic == "split_f16"
        for m in (self.feature_encoder, self.cost_volume_reg, self.depthmap_refine):
            m.split_f16 = split
        return self

    def forward(self, nn_input, K_batch, R_batch, T_batch, d_min, d_int, batch_size, n_views):
        if self._pipeline_ok(nn_input, d_min, d_int, batch_size):
            return self._forward_pipelined(nn_input, K_batch, R_batch, T_batch, d_min, d_int, batch_size, n_views)
        return self._forward_one(nn_input, K_batch, R_batch, T_batch, d_min, d_int, batch_size, n_views)

    def _pipeline_ok(self, nn_input, d_min, d_int, batch_size):
        """The sample-pipelined eval forward applies: HIP fp32 inference with every module in eval mode
        (samples are then independent: eval BatchNorm is elementwise), at least two samples, and
        pipeline_chunks > 1 (MVS_PIPELINE_CHUNKS; 1 = off)."""
        k = self.pipeline_chunks
        return (k > 1 and int(batch_size) >= 2 and _hip_inference(nn_input) and not self.training
                and not any(m.training for m in self.modules())
                and all(t.numel() == 1 or t.shape[0] == int(batch_size) for t in (d_min, d_int))
                and _uniform_depths(d_min, d_int))

    def _forward_pipelined(self, nn_input, K_batch, R_batch, T_batch, d_min, d_int, batch_size, n_views):
        """forward over the batch in ``pipeline_chunks`` chunks of samples, each issued on its own stream
        (lane): one chunk's encoder and cost volume (VALU / HBM-store bound) run beside another chunk's
        regulariser (matrix cores), instead of the whole batch's phases one after another.  Every kernel of
        the eval forward computes each sample independently, so the depth maps are bit-identical to the
        one-stream forward (tests/test_gpu_parity.py::test_pipelined_forward_is_bit_identical)."""
        B, V = int(batch_size), int(n_views)
        k = min(self.pipeline_chunks, B)
        cuts = [B * i // k for i in range(k + 1)]
        device = nn_input.device
        main = torch.cuda.current_stream(device)
        per = lambda t, b0, b1: t if t.numel() == 1 else t[b0:b1]
        outs = []
        for i in range(k):
            b0, b1 = cuts[i], cuts[i + 1]
            st = _lane_stream(device, i)
            st.wait_stream(main)
            _LANE[0] = i + 1
            try:
                with torch.cuda.stream(st):
                    outs.append((st,) + self._forward_one(
                        nn_input[b0 * V:b1 * V], K_batch[b0 * V:b1 * V], R_batch[b0 * V:b1 * V],
                        T_batch[b0 * V:b1 * V], per(d_min, b0, b1), per(d_int, b0, b1), b1 - b0, V))
            finally:
                _LANE[0] = 0
        for st, ini, ref in outs:
            main.wait_stream(st)
            ini.record_stream(main)
            ref.record_stream(main)
        return torch.cat([o[1] for o in outs]), torch.cat([o[2] for o in outs])

    def _forward_one(self, nn_input, K_batch, R_batch, T_batch, d_min, d_int, batch_size, n_views):
        c = self.cfg
        device = nn_input.device
        feature_maps = self.feature_encoder(nn_input)
        bf16 = c.cv_dtype == "bfloat16"
        reg = self.cost_volume_reg
        # HIP inference on the live paths: the cost volume goes straight to the regulariser's kernels
        # in the channel-quad layout (ops.cost_volume_c4: the fused kernel's 16-byte store; with the
        # bf16 opt-in ops.cost_volume_c4_bf16, 8 bytes)
        quads = (_hip_inference(feature_maps) and 2 <= n_views <= 8
                 and feature_maps.shape[1] % 4 == 0
                 and (reg.live_ok((c.d_num,) + tuple(feature_maps.shape[2:]))
                      or reg.live_train_ok((c.d_num,) + tuple(feature_maps.shape[2:]))))
        # eval mode with the split-fp16 regulariser: the fused kernel writes the split cost volume
        # (and in train-mode BN, test.py:61, whose live path reads the split volume the same way)
        live_n = (c.d_num,) + tuple(feature_maps.shape[2:])
        split = (quads and not bf16 and reg.split_f16 and (reg.live_ok(live_n) or reg.live_train_ok(live_n))
                 and feature_maps.shape[1] == 32)
        # ... and with the opt-in fused head kernel (MVS_CV_HEAD=1), the volume is not formed here at
        # all: the regulariser forms it on chip inside conv_0_0 / conv_1_0.  Opt-in:
        # its gathering producers corrupt one item sporadically; the default path
        # materialises the split volume and runs both convolutions in one pass (ops.split_head)
        deferred = split and reg.live_ok(live_n) and (c.d_num % 2 == 0 and n_views in (2, 3)
                                                      and all(p % 2 == 1 for p in reg.pad)
                                                      and os.environ.get("MVS_CV_HEAD", "0") == "1")
        cost_volume, d_batch, ref_views = warp_and_assemble_cost_volume(
            K_batch, R_batch, T_batch, d_min, d_int, feature_maps, batch_size, n_views,
            d_num=c.d_num, d_scale=c.d_scale,
            cv_dtype=torch.bfloat16 if bf16 else torch.float32, channel_quads=quads and not deferred,
            split=split, deferred=deferred)
        if bf16 and not quads:
            # opt-in: the volume is STORED in bf16 (rounded once); the regulariser
            # computes in fp32 from the rounded values, as the HIP channel-quad path does
            cost_volume = cost_volume.float()
        prob_volume = self.cost_volume_reg(cost_volume)
        initial_depth_map = extract_depth_map(prob_volume, d_batch, c.n_depth_est)
        return initial_depth_map, self.refine(nn_input, initial_depth_map, d_min, d_int, ref_views)

    def refine(self, nn_input, initial_depth_map, d_min, d_int, ref_views):
        """model.py:189-205: normalise, concat the downsampled reference image, refine, rescale."""
        c = self.cfg
        device = initial_depth_map.device
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            ref_img = F.interpolate(_select_images(nn_input, ref_views), (c.feat_h, c.feat_w), mode="bilinear")
        if (_hip_inference(initial_depth_map) and initial_depth_map.dim() == 4 and initial_depth_map.shape[1] == 1
                and tuple(ref_img.shape) == (initial_depth_map.shape[0], 3) + tuple(initial_depth_map.shape[2:])
                and all(t.numel() == 1 or tuple(t.shape) == (initial_depth_map.shape[0], 1, 1, 1)
                        for t in (d_min, d_int))   # per sample [B, 1, 1, 1] (data.py) or one value
                and os.environ.get("MVS_REFINE_GLUE", "1") != "0"):
            # the elementwise steps on either side of the refinement net as one HIP launch each
            # (ops.refine_input / refine_output: 9 launches -> 2, bit-equal to the sequence below)
            from .ops import refine_input, refine_output
            x = refine_input(initial_depth_map, d_min, d_int, c.d_num, c.d_scale, ref_img)
            return refine_output(_run_stack(self.depthmap_refine.model, x, self.depthmap_refine.split_f16), x,
                                 d_min, d_int, c.d_num, c.d_scale)
        d_trans = d_min.to(device)
        d_span = d_int.to(device).mul(c.d_num).mul(c.d_scale)
        norm_depth = torch.div(torch.subtract(initial_depth_map, d_trans), d_span)
        refined = self.depthmap_refine(torch.cat((norm_depth, ref_img), dim=1))
        return refined.mul(d_span).add(d_trans)
