"""ORACLE / TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference's cost-volume path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / the timed CPU baseline -- never as the product.  The
product path (``mvs_amd``) runs the HIP kernels and fails loudly without them.

Restates, in torch fp32 on the CPU (the reference's own numeric library), with the reference's
op order so that timings and roundings track it:

  * ``depth_planes``        -- ``scripts/homography.py:24-26``  (d_batch_0, view-major tiling quirk)
  * ``view_indices``        -- ``scripts/homography.py:29-36``  (ref_idx_0, ref_idx, img_idx)
  * ``plane_homographies``  -- ``scripts/homography.py:40-75``  (H_i = K_v R_v (I - (C_v-C_r) n^T/d) R_r^T K_r^-1)
  * ``homography_warping``  -- ``scripts/homography.py:6-92``   (per-plane warp loop, torch.cat growth)
  * ``assemble_cost_volume``-- ``scripts/costvolume.py:3-16``   (two-pass population variance over views)
  * ``extract_depth_map``   -- ``scripts/depthmap.py:4-22``     (permutation-indexed "top-N" mask soft-argmin)
  * ``mvsnet_forward``      -- ``scripts/model.py:168-207``     (the forward around the hot path)
  * ``loss_fcn``            -- ``scripts/loss.py:4-41``         (masked MAE of initial + refined depth)
  * ``mvsnet_forward64``    -- ``scripts/model.py:168-207`` in float64 with the float64 cost-volume law
                               (the gradient oracle of the train.py:97-104 step)

Parity pin: ``tests/golden/*.npz`` were produced by importing the reference's own
``homography.py`` / ``costvolume.py`` / ``depthmap.py`` / ``model.py`` (with the kornia 0.6.3
restatement in ``oracle/kornia_warp.py`` standing in for the absent third-party package) --
see ``tests/golden/make_golden.py``; ``tests/test_oracle.py`` checks this module against them.
The kornia internals themselves are "parity unpinned" (see ``oracle/kornia_warp.py``).
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kornia_warp import warp_normalized, warp_perspective  # noqa: E402

D_SCALE = 25      # scripts/config.py:6
N_DEPTH_EST = 5   # scripts/config.py:9


def depth_planes(d_min, d_int, d_num, d_scale=D_SCALE):
    """homography.py:24-26 -> (d_batch_0 [B,D,1,1], d_batch [V*B,D,1,1] after tiling)."""
    k = torch.arange(d_num).reshape(1, d_num, 1, 1)
    return d_min + d_scale * d_int * k


def view_indices(batch_size, n_views):
    """homography.py:29-36.  ref of image i is n_views*floor(i/n_views); every image warps."""
    n = batch_size * n_views
    ref_idx_0 = torch.arange(0, n, n_views)
    ref_idx, _ = torch.sort(torch.tile(ref_idx_0, (1, n_views)))
    return ref_idx_0, ref_idx.squeeze(0), torch.arange(0, n)


def plane_homographies(K, R, T, d_batch, ref_idx, img_idx, d_num):
    """homography.py:40-75 with the same factorisation and product order, fp32.

    K, R: [N,3,3]; T: [N,3,1]; d_batch: [N,D,1,1] (row i uses sample i mod B).
    Returns H [N,D,3,3] mapping reference pixels to view pixels."""
    rep = lambda m: m.unsqueeze(1).repeat(1, d_num, 1, 1)
    eye = torch.eye(3).unsqueeze(0).unsqueeze(1).repeat(1, d_num, 1, 1)
    K_r, R_r0, T_r0 = K[ref_idx], R[ref_idx], T[ref_idx]
    K_v, R_v0, T_v0 = K[img_idx], R[img_idx], T[img_idx]
    R_r = rep(R_r0)
    C_r = rep(-torch.matmul(R_r0.transpose(-2, -1), T_r0))     # camera centre of the ref view
    n_r = R_r[:, :, :, 2].unsqueeze(2)                         # 3rd column of R_ref, as a row
    R_v = rep(R_v0)
    C_v = rep(-torch.matmul(R_v0.transpose(-2, -1), T_v0))
    left = torch.matmul(rep(K_v), R_v)                         # {1}
    right = torch.matmul(R_r.transpose(-2, -1), torch.inverse(rep(K_r)))   # {3}
    plane = eye - torch.matmul(C_v - C_r, n_r) / d_batch       # {2}
    return torch.matmul(left, torch.matmul(plane, right))


def sampling_matrices64(K_batch, R_batch, T_batch, d_min, d_int, batch_size, n_views, d_num, h, w,
                        d_scale=D_SCALE):
    """The per-(image, plane) normalised sampling matrix ``G = inv(N H N^-1)`` that kornia's
    ``warp_perspective`` forms (homography.py:40-75 for H, kornia 0.6.3 ``normalize_homography`` +
    ``inverse``), composed and inverted in FLOAT64 instead of the reference's fp32 -- the planes
    themselves are the reference's fp32 ``d_batch`` (homography.py:24-26).  Returns float64
    [N, D, 3, 3].  Used by ``homography_warping(..., hom64=True)`` to separate the reference's fp32
    homography rounding from the rest of its arithmetic (tests/golden/make_cfg5_oracle.py)."""
    d_batch = torch.tile(depth_planes(d_min, d_int, d_num, d_scale), (n_views, 1, 1, 1))
    _, ref_idx, img_idx = view_indices(batch_size, n_views)
    H = plane_homographies(K_batch.double(), R_batch.double(), T_batch.double(), d_batch.double(),
                           ref_idx, img_idx, d_num)
    n_src = torch.tensor([[2.0 / (w - 1), 0.0, -1.0], [0.0, 2.0 / (h - 1), -1.0], [0.0, 0.0, 1.0]],
                         dtype=torch.float64)
    return torch.inverse(n_src @ (H @ torch.inverse(n_src)))


def homography_warping(K_batch, R_batch, T_batch, d_min, d_int, feature_maps, batch_size,
                       n_views, d_num, d_scale=D_SCALE, concat_growth=True, hom64=False):
    """homography.py:6-92 restated.  Returns (warped [N,C,D,h,w], d_batch_0 [B,D,1,1], ref_idx_0).

    ``concat_growth=True`` keeps the reference's O(D^2) ``torch.cat`` accumulation (:83-90) -- the
    timed CPU baseline; ``False`` stacks the same per-plane results (same values, test speed).
    ``hom64=True`` (NOT the reference: a diagnostic variant) samples through the float64-composed
    sampling matrices rounded once to fp32 (``sampling_matrices64``), everything after them -- the
    meshgrid, ``transform_points``, ``grid_sample`` -- the reference's fp32 ops unchanged."""
    d_batch_0 = depth_planes(d_min, d_int, d_num, d_scale)
    d_batch = torch.tile(d_batch_0, (n_views, 1, 1, 1))
    ref_idx_0, ref_idx, img_idx = view_indices(batch_size, n_views)
    hw = tuple(feature_maps.shape[-2:])
    if hom64:
        G = sampling_matrices64(K_batch, R_batch, T_batch, d_min, d_int, batch_size, n_views, d_num,
                                hw[0], hw[1], d_scale).float()
    else:
        H = plane_homographies(K_batch.float(), R_batch.float(), T_batch.float(), d_batch,
                               ref_idx, img_idx, d_num)
    src = feature_maps[img_idx]
    planes = []
    warped = None
    for k in range(d_num):
        if hom64:
            cur = warp_normalized(src, G[:, k], hw, align_corners=False).unsqueeze(2)
        else:
            cur = warp_perspective(src, H[:, k], hw, align_corners=False).unsqueeze(2)
        if concat_growth:
            warped = cur if warped is None else torch.cat((warped, cur), 2)
        else:
            planes.append(cur)
    if not concat_growth:
        warped = torch.cat(planes, 2)
    return warped, d_batch_0, ref_idx_0


def assemble_cost_volume(warped, n_views):
    """costvolume.py:3-16: cv = sum_v (x_v - mean)^2 / V with mean = sum_v x_v / V."""
    bn, c, d, h, w = warped.shape
    x = warped.reshape(bn // n_views, n_views, c, d, h, w)
    mean = (x.sum(1) / n_views).unsqueeze(1)
    return (x - mean).pow(2).sum(1) / n_views


def extract_depth_map(prob_volume, d_batch, n_est=N_DEPTH_EST):
    """depthmap.py:4-22: mask[r] = argsort_desc(P)[r] < n_est, depth = sum d P mask / sum P mask."""
    _, order = prob_volume.sort(2, descending=True)
    keep = torch.less(order, torch.tensor(n_est)).float()
    filt = prob_volume * keep
    return (d_batch.unsqueeze(1) * filt).sum(2).squeeze(2).div(filt.sum(2))


def mvsnet_forward(model, nn_input, K_batch, R_batch, T_batch, d_min, d_int, batch_size, n_views,
                   d_num, feat_hw, d_scale=D_SCALE, concat_growth=False, hom64=False):
    """model.py:168-207 on the CPU with the oracle hot path.  ``model`` supplies the three nn
    sub-modules (feature_encoder, cost_volume_reg, depthmap_refine) -- plain torch layers.
    ``hom64``: see ``homography_warping`` (diagnostic variant, not the reference)."""
    feats = model.feature_encoder(nn_input)
    warped, d_batch, ref_views = homography_warping(K_batch, R_batch, T_batch, d_min, d_int, feats,
                                                    batch_size, n_views, d_num, d_scale,
                                                    concat_growth=concat_growth, hom64=hom64)
    cv = assemble_cost_volume(warped, n_views)
    reg = model.cost_volume_reg
    # the reference's op sequence (model.py:100-126) over the whole volume: the build's
    # eval-mode live-region shortcut (CostVolumeReg.forward_live) is not the oracle
    prob = reg.forward_full(cv) if hasattr(reg, "forward_full") else reg(cv)
    initial = extract_depth_map(prob, d_batch)
    d_trans = d_min
    d_span = d_int.mul(d_num).mul(d_scale)
    norm = torch.div(torch.subtract(initial, d_trans), d_span)
    refine_in = torch.cat((norm, F.interpolate(nn_input[ref_views], feat_hw, mode="bilinear")), dim=1)
    refined = model.depthmap_refine(refine_in).mul(d_span).add(d_trans)
    return initial, refined, prob


def loss_fcn(gt, initial, refined):
    """loss.py:4-41: mask = gt != 0; per sample the masked mean absolute error of the initial and of
    the refined depth map (sum over the map / valid pixels); loss = sum over samples of both;
    accuracies = the per-sample MAEs averaged over the batch."""
    mask = torch.ne(gt, torch.tensor(0.0, dtype=gt.dtype, device=gt.device)).to(gt.dtype)
    p_valid = mask.sum((1, 2, 3))
    initial_diff = torch.abs(torch.subtract(gt, initial))
    refined_diff = torch.abs(torch.subtract(gt, refined))
    loss_0 = torch.multiply(mask, initial_diff).sum((1, 2, 3)).div(p_valid)
    loss_1 = torch.multiply(mask, refined_diff).sum((1, 2, 3)).div(p_valid)
    return (loss_0 + loss_1).sum(), loss_0.mean(), loss_1.mean()


def mvsnet_forward64(model, nn_input, K_batch, R_batch, T_batch, d_min, d_int, batch_size, n_views,
                     d_num, feat_hw, d_scale=D_SCALE):
    """model.py:168-207 in float64 on the CPU: ``model`` converted with ``.double()``, the cost
    volume by the float64 law (``cost_volume_torch64``: differentiable in the features, free of the
    reference's fp32 homography noise), the reference's regulariser op sequence, soft-argmin and
    refinement in float64.  The gradient oracle of the training step (train.py:97-104)."""
    x = nn_input.double()
    feats = model.feature_encoder(x)
    cv = cost_volume_torch64(feats, K_batch, R_batch, T_batch, d_min, d_int, batch_size, n_views, d_num,
                             d_scale)
    reg = model.cost_volume_reg
    prob = reg.forward_full(cv) if hasattr(reg, "forward_full") else reg(cv)
    d_batch = depth_planes(d_min.double(), d_int.double(), d_num, d_scale)
    initial = extract_depth_map(prob, d_batch)
    d_trans = d_min.double()
    d_span = d_int.double().mul(d_num).mul(d_scale)
    norm = torch.div(torch.subtract(initial, d_trans), d_span)
    ref_views = view_indices(batch_size, n_views)[0]
    refine_in = torch.cat((norm, F.interpolate(x[ref_views], feat_hw, mode="bilinear")), dim=1)
    refined = model.depthmap_refine(refine_in).mul(d_span).add(d_trans)
    return initial, refined, prob


# ---------------------------------------------------------------------------------------------
# Independent float64 restatement (numpy) of the fused path: the analytic sampling law
# ix = xs*w/(w-1) - 0.5 with xs = dehom(H^-1 [x,y,1]), used by the known-answer
# tests to cross-check the torch restatement above without going through kornia's matrices.
# ---------------------------------------------------------------------------------------------
def sample_bilinear_zero_np(img, ix, iy):
    """grid_sample(bilinear, zeros, align_corners=False) at absolute source coords (float64)."""
    c, h, w = img.shape
    x0 = np.floor(ix)
    y0 = np.floor(iy)
    out = np.zeros((c,) + ix.shape, dtype=np.float64)
    for dy in (0, 1):
        for dx in (0, 1):
            xx = x0 + dx
            yy = y0 + dy
            wgt = (1.0 - np.abs(ix - xx)) * (1.0 - np.abs(iy - yy))
            ok = (xx >= 0) & (xx < w) & (yy >= 0) & (yy < h)
            xi = np.where(ok, xx, 0).astype(np.int64)
            yi = np.where(ok, yy, 0).astype(np.int64)
            out += np.where(ok, wgt, 0.0)[None] * img[:, yi, xi]
    return out


def cost_volume_fp64(feat, K, R, T, d_min, d_int, batch_size, n_views, d_num, d_scale=D_SCALE,
                     d_begin=0, d_count=None):
    """float64 numpy cost volume [B,C,d_count,h,w] by the analytic law (no kornia matrices)."""
    feat = np.asarray(feat, np.float64)
    K = np.asarray(K, np.float64)
    R = np.asarray(R, np.float64)
    T = np.asarray(T, np.float64).reshape(-1, 3, 1)
    d_min = np.asarray(d_min, np.float64).reshape(-1)
    d_int = np.asarray(d_int, np.float64).reshape(-1)
    n, c, h, w = feat.shape
    if d_count is None:
        d_count = d_num - d_begin
    ys, xs = np.meshgrid(np.arange(h, dtype=np.float64), np.arange(w, dtype=np.float64), indexing="ij")
    pix = np.stack([xs.ravel(), ys.ravel(), np.ones(h * w)])
    cv = np.zeros((batch_size, c, d_count, h, w))
    for b in range(batch_size):
        r = b * n_views
        C_r = -R[r].T @ T[r]
        n_r = R[r][:, 2:3].T
        for kk in range(d_count):
            k = d_begin + kk
            vals = []
            for v in range(n_views):
                i = b * n_views + v
                d = d_min[i % batch_size] + d_scale * d_int[i % batch_size] * k
                C_i = -R[i].T @ T[i]
                H = K[i] @ R[i] @ (np.eye(3) - (C_i - C_r) @ n_r / d) @ R[r].T @ np.linalg.inv(K[r])
                src = np.linalg.inv(H) @ pix
                s = src[2]
                good = np.abs(s) > 1e-8
                sx = np.where(good, src[0] / np.where(good, s, 1.0), src[0])
                sy = np.where(good, src[1] / np.where(good, s, 1.0), src[1])
                # kornia normalises with (w-1), grid_sample(align_corners=False) unnormalises with w
                ix = sx * w / (w - 1) - 0.5
                iy = sy * h / (h - 1) - 0.5
                vals.append(sample_bilinear_zero_np(feat[i], ix.reshape(h, w), iy.reshape(h, w)))
            x = np.stack(vals)
            cv[b, :, kk] = ((x - x.mean(0)) ** 2).mean(0)
    return cv


def cost_volume_torch64(feat, K, R, T, d_min, d_int, batch_size, n_views, d_num, d_scale=D_SCALE,
                        d_begin=0, d_count=None):
    """The float64 law of ``cost_volume_fp64`` in torch (differentiable w.r.t. ``feat``): the
    gradient oracle for the backward, free of the reference's fp32 homography noise.  Sampling at
    ix = xs*w/(w-1) - 0.5 (xs = dehom(H^-1 [x,y,1])) through grid_sample(bilinear, zeros,
    align_corners=False) with the normalised coordinate (2 ix + 1) / w - 1."""
    feat = torch.as_tensor(feat).double()
    K = np.asarray(K, np.float64)
    R = np.asarray(R, np.float64)
    T = np.asarray(T, np.float64).reshape(-1, 3, 1)
    d_min = np.asarray(d_min, np.float64).reshape(-1)
    d_int = np.asarray(d_int, np.float64).reshape(-1)
    n, c, h, w = feat.shape
    if d_count is None:
        d_count = d_num - d_begin
    ys, xs = np.meshgrid(np.arange(h, dtype=np.float64), np.arange(w, dtype=np.float64), indexing="ij")
    pix = np.stack([xs.ravel(), ys.ravel(), np.ones(h * w)])
    out = []
    for b in range(batch_size):
        r = b * n_views
        C_r = -R[r].T @ T[r]
        n_r = R[r][:, 2:3].T
        grids = []
        for v in range(n_views):
            i = b * n_views + v
            C_i = -R[i].T @ T[i]
            gv = []
            for kk in range(d_count):
                d = d_min[i % batch_size] + d_scale * d_int[i % batch_size] * (d_begin + kk)
                H = K[i] @ R[i] @ (np.eye(3) - (C_i - C_r) @ n_r / d) @ R[r].T @ np.linalg.inv(K[r])
                src = np.linalg.inv(H) @ pix
                s = src[2]
                good = np.abs(s) > 1e-8
                sx = np.where(good, src[0] / np.where(good, s, 1.0), src[0])
                sy = np.where(good, src[1] / np.where(good, s, 1.0), src[1])
                ix = sx * w / (w - 1) - 0.5
                iy = sy * h / (h - 1) - 0.5
                gv.append(np.stack([(2 * ix + 1) / w - 1, (2 * iy + 1) / h - 1], -1).reshape(h, w, 2))
            grids.append(torch.from_numpy(np.stack(gv)))          # [D, h, w, 2]
        x = torch.stack([F.grid_sample(feat[b * n_views + v].unsqueeze(0).expand(d_count, c, h, w),
                                       grids[v], mode="bilinear", padding_mode="zeros",
                                       align_corners=False) for v in range(n_views)])   # [V, D, C, h, w]
        mean = x.mean(0, keepdim=True)
        out.append(((x - mean) ** 2).mean(0).permute(1, 0, 2, 3))   # [C, D, h, w]
    return torch.stack(out)
