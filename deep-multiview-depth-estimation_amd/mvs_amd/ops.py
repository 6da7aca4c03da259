"""torch.library custom ops over the C ABI (namespace ``mvs``), with autograd and fake kernels.

  mvs::cost_volume            fused warp + variance      (homography.py:6-92 + costvolume.py:3-16)
  mvs::cost_volume_bf16       same, bf16 cost volume     (opt-in)
  mvs::cost_volume_c4         same, channel-quad layout  (inference feed of the HIP regulariser)
  mvs::cost_volume_c4_bf16    same, bf16 channel-quad    (SURVEY.md §8 f3 opt-in inference feed)
  mvs::cost_volume_backward   d cv / d feat              (autograd of the above, train.py:103)
  mvs::homography_warp        warp only                  (homography.py:6-92 warped volume)
  mvs::assemble_cost_volume   variance of a warped volume (costvolume.py:3-16)
  mvs::extract_depth_map      masked soft-argmin          (depthmap.py:4-22)

Every op requires CUDA(HIP) tensors and raises otherwise: there is no CPU path in the product.
Camera tensors (K, R, T, d_min, d_int) are moved to the feature device here, as the reference
does with ``.to(DEVICE)`` (homography.py:25,43-58).
"""
import ctypes
import weakref
from typing import Optional

import torch

from . import _lib

_F32 = torch.float32


def _require_gpu(t, name):
    if not t.is_cuda:
        raise _lib.MVSLibraryError(
            "%s must be a GPU (HIP) tensor: the MI355X cost-volume path has no CPU fallback" % name)


def _eager_only(op, **side_outputs):
    """Fake-kernel guard of the ops that raise bound words / write batch sums IN PLACE without declaring
    the mutation (mutates_args=(): torch's ADInplaceOrView wrapper cannot index an omitted trailing
    optional): under torch.compile / functionalization such writes could be reordered or dropped, so a
    trace that passes one fails here instead.  Eager mode (what MVSNet runs) is the only valid mode."""
    given = [k for k, v in side_outputs.items() if v is not None]
    if given:
        raise NotImplementedError("mvs::%s writes %s in place (an undeclared mutation): eager mode only, not "
                                  "torch.compile / functionalization" % (op, ", ".join(given)))


def _cams(K, R, T, d_min, d_int, device, batch_size):
    K = K.to(device=device, dtype=_F32).reshape(-1, 3, 3).contiguous()
    R = R.to(device=device, dtype=_F32).reshape(-1, 3, 3).contiguous()
    T = T.to(device=device, dtype=_F32).reshape(-1, 3).contiguous()
    d_min = d_min.to(device=device, dtype=_F32).reshape(-1)
    d_int = d_int.to(device=device, dtype=_F32).reshape(-1)
    if d_min.numel() == 1:
        d_min = d_min.expand(batch_size)
    if d_int.numel() == 1:
        d_int = d_int.expand(batch_size)
    return K, R, T, d_min.contiguous(), d_int.contiguous()


def _check_geometry(feat, K, batch_size, n_views):
    if feat.dim() != 4:
        raise ValueError("feature maps must be [B*V, C, h, w], got %s" % (tuple(feat.shape),))
    n = batch_size * n_views
    if feat.shape[0] != n:
        raise ValueError("feature maps hold %d images, batch_size*n_views = %d" % (feat.shape[0], n))
    if K.shape[0] != n:
        raise ValueError("K holds %d cameras, batch_size*n_views = %d" % (K.shape[0], n))


# ----------------------------------------------------------------------------------------------
# mvs::cost_volume (+ backward)
# ----------------------------------------------------------------------------------------------
@torch.library.custom_op("mvs::cost_volume", mutates_args=())
def cost_volume(feat: torch.Tensor, K: torch.Tensor, R: torch.Tensor, T: torch.Tensor,
                d_min: torch.Tensor, d_int: torch.Tensor, batch_size: int, n_views: int,
                d_begin: int, d_count: int, d_scale: float) -> tuple[torch.Tensor, torch.Tensor]:
    """Fused warp + variance: returns (cv [B,C,d_count,h,w], workspace).  The workspace starts
    with the per-(image, plane) sampling matrices the backward reuses."""
    _require_gpu(feat, "feature_maps")
    lib = _lib.load()
    feat = feat.to(_F32).contiguous()
    K, R, T, d_min, d_int = _cams(K, R, T, d_min, d_int, feat.device, batch_size)
    _check_geometry(feat, K, batch_size, n_views)
    n, c, h, w = feat.shape
    cv = torch.empty((batch_size, c, d_count, h, w), device=feat.device, dtype=_F32)
    ws_bytes = lib.mvs_cost_volume_workspace_bytes(batch_size, n_views, c, h, w, d_count)
    ws = torch.empty((max(ws_bytes, 4) // 4,), device=feat.device, dtype=_F32)
    st = lib.mvs_cost_volume_fwd(_lib.ptr(feat), _lib.ptr(K), _lib.ptr(R), _lib.ptr(T),
                                 _lib.ptr(d_min), _lib.ptr(d_int), batch_size, n_views, c, h, w,
                                 d_begin, d_count, float(d_scale), _lib.ptr(ws), _lib.ptr(cv),
                                 _lib.stream_handle(feat.device))
    _lib.check(st, "mvs_cost_volume_fwd")
    return cv, ws


def _ws_floats(batch_size, n_views, c, h, w, d_count):
    """Workspace size in floats, from the library's own size function (host-only, no GPU)."""
    return max(_lib.load().mvs_cost_volume_workspace_bytes(batch_size, n_views, c, h, w, d_count), 4) // 4


@cost_volume.register_fake
def _(feat, K, R, T, d_min, d_int, batch_size, n_views, d_begin, d_count, d_scale):
    n, c, h, w = feat.shape
    return (feat.new_empty((batch_size, c, d_count, h, w)),
            feat.new_empty((_ws_floats(batch_size, n_views, c, h, w, d_count),)))


@torch.library.custom_op("mvs::cost_volume_bf16", mutates_args=())
def cost_volume_bf16(feat: torch.Tensor, K: torch.Tensor, R: torch.Tensor, T: torch.Tensor,
                     d_min: torch.Tensor, d_int: torch.Tensor, batch_size: int, n_views: int,
                     d_begin: int, d_count: int, d_scale: float) -> tuple[torch.Tensor, torch.Tensor]:
    """mvs::cost_volume with a bf16 cost volume (opt-in): the fp32 variance
    rounded to nearest-even in the kernel's store, half the HBM write."""
    _require_gpu(feat, "feature_maps")
    lib = _lib.load()
    feat = feat.to(_F32).contiguous()
    K, R, T, d_min, d_int = _cams(K, R, T, d_min, d_int, feat.device, batch_size)
    _check_geometry(feat, K, batch_size, n_views)
    n, c, h, w = feat.shape
    cv = torch.empty((batch_size, c, d_count, h, w), device=feat.device, dtype=torch.bfloat16)
    ws = torch.empty((_ws_floats(batch_size, n_views, c, h, w, d_count),), device=feat.device,
                     dtype=_F32)
    st = lib.mvs_cost_volume_fwd_bf16(_lib.ptr(feat), _lib.ptr(K), _lib.ptr(R), _lib.ptr(T),
                                      _lib.ptr(d_min), _lib.ptr(d_int), batch_size, n_views, c, h, w,
                                      d_begin, d_count, float(d_scale), _lib.ptr(ws), _lib.ptr(cv),
                                      _lib.stream_handle(feat.device))
    _lib.check(st, "mvs_cost_volume_fwd_bf16")
    return cv, ws


@cost_volume_bf16.register_fake
def _(feat, K, R, T, d_min, d_int, batch_size, n_views, d_begin, d_count, d_scale):
    n, c, h, w = feat.shape
    return (feat.new_empty((batch_size, c, d_count, h, w), dtype=torch.bfloat16),
            feat.new_empty((_ws_floats(batch_size, n_views, c, h, w, d_count),)))


# Live timing of the main fused kernel inside a real step (bench.py): when set, a callable returning a
# KERNEL_EVENT_HOOK(kind) -> (begin, end) pair of torch.cuda.Event for each fused-kernel call (kind
# "cost_volume": the cost_volume_c4* ops' warp kernel; "split_head": ops.split_head; "cv_head": the
# opt-in fused head); the C ABI records them on the launch stream right around that kernel (the ops'
# event arguments).
KERNEL_EVENT_HOOK = None


class timed_kernel:
    """``with timed_kernel("conv_0_0"):`` -- KERNEL_EVENT_HOOK's event pair recorded on the CURRENT stream
    right before and after the block (which launches one kernel on that stream, e.g. conv3d_k3); a
    no-op when no hook is set."""

    def __init__(self, kind):
        self.kind, self.pair = kind, None

    def __enter__(self):
        if KERNEL_EVENT_HOOK is not None:
            self.pair = KERNEL_EVENT_HOOK(self.kind)
            self.pair[0].record(torch.cuda.current_stream())
        return self

    def __exit__(self, *exc):
        if self.pair is not None:
            self.pair[1].record(torch.cuda.current_stream())
        return False


@torch.library.custom_op("mvs::cost_volume_c4", mutates_args=())
def cost_volume_c4(feat: torch.Tensor, K: torch.Tensor, R: torch.Tensor, T: torch.Tensor,
                   d_min: torch.Tensor, d_int: torch.Tensor, batch_size: int, n_views: int,
                   d_begin: int, d_count: int, d_scale: float) -> torch.Tensor:
    """mvs::cost_volume in the channel-quad layout cv[B][C/4][d_count][h][w][4] (the same values:
    cv_c4[b, q, d, y, x, j] == cv[b, 4q + j, d, y, x]), what conv3d_k3 / conv3d_region (CONV_S2)
    read with in_c4=True.  Inference only (no autograd formula), 2 <= n_views <= 8, C % 4 == 0."""
    _require_gpu(feat, "feature_maps")
    lib = _lib.load()
    feat = feat.to(_F32).contiguous()
    K, R, T, d_min, d_int = _cams(K, R, T, d_min, d_int, feat.device, batch_size)
    _check_geometry(feat, K, batch_size, n_views)
    n, c, h, w = feat.shape
    if c % 4:
        raise ValueError("the channel-quad cost volume needs C % 4 == 0, got C=%d" % c)
    cv = torch.empty((batch_size, c // 4, d_count, h, w, 4), device=feat.device, dtype=_F32)
    ws = torch.empty((_ws_floats(batch_size, n_views, c, h, w, d_count),), device=feat.device,
                     dtype=_F32)
    evs = (None, None)
    if KERNEL_EVENT_HOOK is not None:
        evs = tuple(ctypes.c_void_p(e.cuda_event) for e in KERNEL_EVENT_HOOK("cost_volume"))
    st = lib.mvs_cost_volume_fwd_c4(_lib.ptr(feat), _lib.ptr(K), _lib.ptr(R), _lib.ptr(T),
                                    _lib.ptr(d_min), _lib.ptr(d_int), batch_size, n_views, c, h, w,
                                    d_begin, d_count, float(d_scale), _lib.ptr(ws), _lib.ptr(cv),
                                    _lib.stream_handle(feat.device), *evs)
    _lib.check(st, "mvs_cost_volume_fwd_c4")
    return cv


@cost_volume_c4.register_fake
def _(feat, K, R, T, d_min, d_int, batch_size, n_views, d_begin, d_count, d_scale):
    n, c, h, w = feat.shape
    return feat.new_empty((batch_size, c // 4, d_count, h, w, 4))


@torch.library.custom_op("mvs::cost_volume_c4_absmax", mutates_args=())
def cost_volume_c4_absmax(feat: torch.Tensor, K: torch.Tensor, R: torch.Tensor, T: torch.Tensor,
                          d_min: torch.Tensor, d_int: torch.Tensor, batch_size: int, n_views: int,
                          d_begin: int, d_count: int, d_scale: float) -> tuple[torch.Tensor, torch.Tensor]:
    """cost_volume_c4 plus its bound words (mvs_cost_volume_fwd_c4_absmax): absmax int32[8] holds the
    per-XCD maxima of the |feat| bit patterns, every cost-volume element is <= (the largest, as a
    float)^2 -- what the split-fp16 conv_0_0 (conv3d_k3_split) scales its operands by."""
    _require_gpu(feat, "feature_maps")
    lib = _lib.load()
    feat = feat.to(_F32).contiguous()
    K, R, T, d_min, d_int = _cams(K, R, T, d_min, d_int, feat.device, batch_size)
    _check_geometry(feat, K, batch_size, n_views)
    n, c, h, w = feat.shape
    if c % 4:
        raise ValueError("the channel-quad cost volume needs C % 4 == 0, got C=%d" % c)
    cv = torch.empty((batch_size, c // 4, d_count, h, w, 4), device=feat.device, dtype=_F32)
    absmax = torch.empty((8,), device=feat.device, dtype=torch.int32)
    ws = torch.empty((_ws_floats(batch_size, n_views, c, h, w, d_count),), device=feat.device,
                     dtype=_F32)
    evs = (None, None)
    if KERNEL_EVENT_HOOK is not None:
        evs = tuple(ctypes.c_void_p(e.cuda_event) for e in KERNEL_EVENT_HOOK("cost_volume"))
    st = lib.mvs_cost_volume_fwd_c4_absmax(_lib.ptr(feat), _lib.ptr(K), _lib.ptr(R), _lib.ptr(T),
                                           _lib.ptr(d_min), _lib.ptr(d_int), batch_size, n_views, c, h, w,
                                           d_begin, d_count, float(d_scale), _lib.ptr(ws), _lib.ptr(cv),
                                           _lib.stream_handle(feat.device), *evs, _lib.ptr(absmax))
    _lib.check(st, "mvs_cost_volume_fwd_c4_absmax")
    return cv, absmax


@cost_volume_c4_absmax.register_fake
def _(feat, K, R, T, d_min, d_int, batch_size, n_views, d_begin, d_count, d_scale):
    n, c, h, w = feat.shape
    return feat.new_empty((batch_size, c // 4, d_count, h, w, 4)), feat.new_empty((8,), dtype=torch.int32)


@torch.library.custom_op("mvs::cost_volume_c4_split", mutates_args=())
def cost_volume_c4_split(feat: torch.Tensor, K: torch.Tensor, R: torch.Tensor, T: torch.Tensor,
                         d_min: torch.Tensor, d_int: torch.Tensor, batch_size: int, n_views: int,
                         d_begin: int, d_count: int, d_scale: float) -> tuple[torch.Tensor, torch.Tensor]:
    """The SPLIT cost volume (mvs_cost_volume_fwd_c4_split, csrc/split.h): int32 [B, C/4, d_count, h, w, 4]
    holding, per 16-byte element, the fp16 hi / lo parts of 4 variances scaled by 2^e (e from the bound
    words, returned beside it) -- the operands the split-fp16 regulariser kernels read without
    converting.  unsplit_cost_volume() gives the fp32 values back (to 2^-22)."""
    _require_gpu(feat, "feature_maps")
    lib = _lib.load()
    feat = feat.to(_F32).contiguous()
    K, R, T, d_min, d_int = _cams(K, R, T, d_min, d_int, feat.device, batch_size)
    _check_geometry(feat, K, batch_size, n_views)
    n, c, h, w = feat.shape
    if c % 4:
        raise ValueError("the channel-quad cost volume needs C % 4 == 0, got C=%d" % c)
    cv = torch.empty((batch_size, c // 4, d_count, h, w, 4), device=feat.device, dtype=torch.int32)
    absmax = torch.empty((8,), device=feat.device, dtype=torch.int32)
    ws = torch.empty((_ws_floats(batch_size, n_views, c, h, w, d_count),), device=feat.device,
                     dtype=_F32)
    evs = (None, None)
    if KERNEL_EVENT_HOOK is not None:
        evs = tuple(ctypes.c_void_p(e.cuda_event) for e in KERNEL_EVENT_HOOK("cost_volume"))
    st = lib.mvs_cost_volume_fwd_c4_split(_lib.ptr(feat), _lib.ptr(K), _lib.ptr(R), _lib.ptr(T),
                                          _lib.ptr(d_min), _lib.ptr(d_int), batch_size, n_views, c, h, w,
                                          d_begin, d_count, float(d_scale), _lib.ptr(ws), _lib.ptr(cv),
                                          _lib.stream_handle(feat.device), *evs, _lib.ptr(absmax))
    _lib.check(st, "mvs_cost_volume_fwd_c4_split")
    return cv, absmax


@cost_volume_c4_split.register_fake
def _(feat, K, R, T, d_min, d_int, batch_size, n_views, d_begin, d_count, d_scale):
    n, c, h, w = feat.shape
    return (feat.new_empty((batch_size, c // 4, d_count, h, w, 4), dtype=torch.int32),
            feat.new_empty((8,), dtype=torch.int32))


def split_exponent(absmax):
    """The scale exponent e of a split cost volume from its bound words (csrc/split.h rule, host side)."""
    import math
    m = int(absmax.to(torch.int64).max().item())
    if m == 0 or m >= 0x7F800000:
        return 0
    b = torch.tensor([m], dtype=torch.int32).view(torch.float32).item()
    return min(max(14 - 2 * math.frexp(b)[1], -120), 120)


def unsplit_cost_volume(cv, absmax):
    """fp32 channel-quad [B, C/4, D, h, w, 4] of a split cost volume: (hi + lo) 2^-e per element."""
    e = split_exponent(absmax)
    halves = cv.contiguous().view(torch.float16).reshape(cv.shape[:-1] + (2, 4)).float()
    return torch.ldexp(halves[..., 0, :] + halves[..., 1, :], torch.tensor(-e, device=cv.device,
                                                                            dtype=torch.float32))


class BoundCostVolume:
    """A channel-quad cost volume together with its bound words (csrc/split.h): ``data`` is the fp32
    channel-quad volume [B, C/4, D, h, w, 4] (cost_volume_c4_absmax) or the split volume (int32,
    cost_volume_c4_split), ``absmax`` its int32[8] bound words (every element <= max|feat|^2; the split
    scale).  The two travel as ONE object, so no copy, view or re-layout of the tensor can separate the
    volume from its scale (CostVolumeReg.forward raises on a bare split tensor).

    ``box_origin`` (3 ints) marks a PARTIAL volume: ``data`` then holds only the box
    [box_origin, box_origin + data.shape[2:5]) of a volume of extent ``dims`` -- what the fused head
    stores (conv_2_0 / conv_3_0's input box); such a volume is read only by the box-aware region conv
    (box_region()), and quads() / to_ncdhw() refuse it."""
    __slots__ = ("data", "absmax", "box_origin", "dims")

    def __init__(self, data: torch.Tensor, absmax: torch.Tensor, box_origin=None, dims=None):
        if data.dim() != 6 or data.dtype not in (_F32, torch.int32):
            raise ValueError("channel-quad cost volume [B, C/4, D, h, w, 4] fp32 or int32 expected")
        if absmax.numel() != 8 or absmax.dtype != torch.int32 or absmax.device != data.device:
            raise ValueError("absmax: int32[8] on the volume's device expected")
        if (box_origin is None) != (dims is None):
            raise ValueError("a partial volume needs both its box origin and the full dims")
        if box_origin is not None:
            box_origin, dims = [int(v) for v in box_origin], [int(v) for v in dims]
            if len(box_origin) != 3 or len(dims) != 3 or any(
                    o < 0 or o + s > d for o, s, d in zip(box_origin, data.shape[2:5], dims)):
                raise ValueError("box %s + %s outside the volume %s" % (box_origin, list(data.shape[2:5]), dims))
        self.data, self.absmax, self.box_origin, self.dims = data, absmax, box_origin, dims

    shape = property(lambda self: self.data.shape)
    dtype = property(lambda self: self.data.dtype)
    device = property(lambda self: self.data.device)
    is_cuda = property(lambda self: self.data.is_cuda)
    split = property(lambda self: self.data.dtype == torch.int32)

    def dim(self):
        return self.data.dim()

    partial = property(lambda self: self.box_origin is not None)

    def clone(self):
        return BoundCostVolume(self.data.clone(), self.absmax.clone(), self.box_origin, self.dims)

    def box_region(self):
        """(origin, size) of the voxels ``data`` holds: the box, or the whole volume."""
        size = [int(v) for v in self.data.shape[2:5]]
        return (list(self.box_origin) if self.partial else [0, 0, 0]), size

    def quads(self):
        """fp32 channel-quad values (the split volume re-formed to 2^-22 relative)."""
        if self.partial:
            raise ValueError("a partial (boxed) cost volume has no values outside its box")
        return unsplit_cost_volume(self.data, self.absmax) if self.split else self.data

    def to_ncdhw(self):
        """The reference layout [B, C, D, h, w] fp32."""
        q = self.quads()
        return q.permute(0, 1, 5, 2, 3, 4).reshape((q.shape[0], 4 * q.shape[1]) + tuple(q.shape[2:5]))


@torch.library.custom_op("mvs::cost_volume_head", mutates_args=())
def cost_volume_head(feat: torch.Tensor, K: torch.Tensor, R: torch.Tensor, T: torch.Tensor,
                     d_min: torch.Tensor, d_int: torch.Tensor, batch_size: int, n_views: int,
                     d_begin: int, d_count: int, d_scale: float, w0: torch.Tensor,
                     bn0_scale: Optional[torch.Tensor], bn0_shift: Optional[torch.Tensor],
                     bn0_mean: Optional[torch.Tensor], w1: torch.Tensor, bn1_scale: Optional[torch.Tensor],
                     bn1_shift: Optional[torch.Tensor], bn1_mean: Optional[torch.Tensor], pad: list[int],
                     y1_origin: list[int], y1_size: list[int], scv_lo: list[int],
                     scv_hi: list[int]) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """The cost volume consumed where it is formed (mvs_cost_volume_head_fwd, csrc/cv_head.hip; SURVEY.md
    §8 f3): warp + variance (homography.py:6-92, costvolume.py:3-16) fused with conv_0_0 + BN_0 + ReLU
    (model.py:101) and conv_1_0 + BN_1 + ReLU (model.py:103) on the split-fp16 matrix cores.  Returns
    (y0 [B, 8, d_count, h, w], y1 channels-last [B, *y1_size, 16], scv, absmax): scv is the split cost
    volume on the box [scv_lo, scv_hi) only (what conv_2_0 / conv_3_0 read), int32
    [B, 8, *(scv_hi - scv_lo), 4]; absmax its bound words.  Bit-identical to cost_volume_c4_split -> conv3d_k3_split /
    conv_s2_split.  C = 32, 2 <= n_views <= 3, d_count even, pad odd; inference only."""
    _require_gpu(feat, "feature_maps")
    lib = _lib.load()
    feat = feat.to(_F32).contiguous()
    K, R, T, d_min, d_int = _cams(K, R, T, d_min, d_int, feat.device, batch_size)
    _check_geometry(feat, K, batch_size, n_views)
    n, c, h, w = feat.shape
    if tuple(w0.shape) != (8, 32, 3, 3, 3) or tuple(w1.shape) != (16, 32, 3, 3, 3):
        raise ValueError("conv_0_0 [8, 32, 3, 3, 3] and conv_1_0 [16, 32, 3, 3, 3] weights expected")
    dev = feat.device
    f0, e0 = derived("k3split", (w0,), lambda wt: split_weight_fragments(wt, dev), dev)
    f1, e1 = derived("s2split", (w1,), lambda wt: _s2_split_fragments(wt, dev), dev)

    def bn(ts):
        ts = [t if t is None else t.to(device=dev, dtype=_F32).contiguous() for t in ts]
        if any(t is None for t in ts) and not all(t is None for t in ts):
            raise ValueError("BN scale, shift and mean go together")
        return ts, [None if t is None else _lib.ptr(t) for t in ts]
    bn0, bp0 = bn((bn0_scale, bn0_shift, bn0_mean))
    bn1, bp1 = bn((bn1_scale, bn1_shift, bn1_mean))
    y0 = torch.empty((batch_size, 8, d_count, h, w), device=dev, dtype=_F32)
    y1 = torch.empty([batch_size] + [int(v) for v in y1_size] + [16], device=dev, dtype=_F32)
    boxed = all(int(hi_) > int(lo_) for lo_, hi_ in zip(scv_lo, scv_hi))
    box = [int(hi_) - int(lo_) for lo_, hi_ in zip(scv_lo, scv_hi)]
    scv = torch.empty([batch_size, 8] + box + [4] if boxed else [0], device=dev, dtype=torch.int32)
    absmax = torch.empty((8,), device=dev, dtype=torch.int32)
    ws = torch.empty((_ws_floats(batch_size, n_views, c, h, w, d_count),), device=dev, dtype=_F32)
    evs = (None, None)
    if KERNEL_EVENT_HOOK is not None:
        evs = tuple(ctypes.c_void_p(e.cuda_event) for e in KERNEL_EVENT_HOOK("cv_head"))
    st = lib.mvs_cost_volume_head_fwd(_lib.ptr(feat), _lib.ptr(K), _lib.ptr(R), _lib.ptr(T), _lib.ptr(d_min),
                                      _lib.ptr(d_int), batch_size, n_views, c, h, w, d_begin, d_count,
                                      float(d_scale), _lib.ptr(f0), int(e0), *bp0, _lib.ptr(f1), int(e1), *bp1,
                                      _ints3(pad), _ints3(y1_origin), _ints3(y1_size), _ints3(scv_lo),
                                      _ints3(scv_hi), _lib.ptr(ws), _lib.ptr(absmax), _lib.ptr(y0), _lib.ptr(y1),
                                      _lib.ptr(scv) if boxed else None, _lib.stream_handle(dev), *evs)
    _lib.check(st, "mvs_cost_volume_head_fwd")
    return y0, y1, scv, absmax


@cost_volume_head.register_fake
def _(feat, K, R, T, d_min, d_int, batch_size, n_views, d_begin, d_count, d_scale, w0, bn0_scale, bn0_shift,
      bn0_mean, w1, bn1_scale, bn1_shift, bn1_mean, pad, y1_origin, y1_size, scv_lo, scv_hi):
    n, c, h, w = feat.shape
    boxed = all(int(hi_) > int(lo_) for lo_, hi_ in zip(scv_lo, scv_hi))
    box = [int(hi_) - int(lo_) for lo_, hi_ in zip(scv_lo, scv_hi)]
    return (feat.new_empty((batch_size, 8, d_count, h, w)), feat.new_empty([batch_size] + list(y1_size) + [16]),
            feat.new_empty([batch_size, 8] + box + [4] if boxed else [0], dtype=torch.int32),
            feat.new_empty((8,), dtype=torch.int32))


# (the bound words are raised in place; not declared as a mutation: torch's ADInplaceOrView wrapper
# indexes every declared mutable argument positionally, which fails for an omitted trailing default)
@torch.library.custom_op("mvs::split_head", mutates_args=())
def split_head(scv: torch.Tensor, absmax: torch.Tensor, w0: torch.Tensor, bn0_scale: Optional[torch.Tensor],
               bn0_shift: Optional[torch.Tensor], bn0_mean: Optional[torch.Tensor], w1: torch.Tensor,
               bn1_scale: Optional[torch.Tensor], bn1_shift: Optional[torch.Tensor], bn1_mean: Optional[torch.Tensor],
               pad: list[int], y1_origin: list[int], y1_size: list[int],
               y1_bound: Optional[torch.Tensor] = None) -> tuple[torch.Tensor, torch.Tensor]:
    """conv_0_0 + BN_0 + ReLU (model.py:101) and conv_1_0 + BN_1 + ReLU (model.py:103) of the split cost
    volume ``scv`` [B, 8, D, h, w, 4] int32 (cost_volume_c4_split) in ONE pass over it
    (mvs_split_head_fwd).  Returns (y0 [B, 8, D, h, w], y1 channels-last [B, *y1_size, 16]): bit-identical
    to conv3d_k3_split and conv_s2_split.  D even, pad odd; inference only.  ``y1_bound``: int32
    [MVS_BOUND_WORDS] zeroed words raised to max|y1| (the scale of conv3d_region_split's input)."""
    _require_gpu(scv, "scv")
    lib = _lib.load()
    if scv.dim() != 6 or scv.dtype != torch.int32 or scv.shape[1] != 8 or scv.shape[5] != 4:
        raise ValueError("split cost volume [B, 8, D, h, w, 4] int32 expected")
    if tuple(w0.shape) != (8, 32, 3, 3, 3) or tuple(w1.shape) != (16, 32, 3, 3, 3):
        raise ValueError("conv_0_0 [8, 32, 3, 3, 3] and conv_1_0 [16, 32, 3, 3, 3] weights expected")
    scv = scv.contiguous()
    b, _, d, h, w, _ = scv.shape
    dev = scv.device
    f0, e0 = derived("k3split", (w0,), lambda wt: split_weight_fragments(wt, dev), dev)
    f1, e1 = derived("s2split", (w1,), lambda wt: _s2_split_fragments(wt, dev), dev)

    def bn(ts):
        ts = [t if t is None else t.to(device=dev, dtype=_F32).contiguous() for t in ts]
        if any(t is None for t in ts) and not all(t is None for t in ts):
            raise ValueError("BN scale, shift and mean go together")
        return ts, [None if t is None else _lib.ptr(t) for t in ts]
    bn0, bp0 = bn((bn0_scale, bn0_shift, bn0_mean))
    bn1, bp1 = bn((bn1_scale, bn1_shift, bn1_mean))
    y0 = torch.empty((b, 8, d, h, w), device=dev, dtype=_F32)
    y1 = torch.empty([b] + [int(v) for v in y1_size] + [16], device=dev, dtype=_F32)
    evs = (None, None)
    if KERNEL_EVENT_HOOK is not None:
        evs = tuple(ctypes.c_void_p(e.cuda_event) for e in KERNEL_EVENT_HOOK("split_head"))
    st = lib.mvs_split_head_fwd(_lib.ptr(scv), _lib.ptr(absmax.contiguous()), b, d, h, w, _lib.ptr(f0), int(e0),
                                *bp0, _lib.ptr(f1), int(e1), *bp1, _ints3(pad), _ints3(y1_origin),
                                _ints3(y1_size), _lib.ptr(y0), _lib.ptr(y1), _bound_ptr(y1_bound),
                                _lib.stream_handle(dev), *evs)
    _lib.check(st, "mvs_split_head_fwd")
    return y0, y1


@split_head.register_fake
def _(scv, absmax, w0, bn0_scale, bn0_shift, bn0_mean, w1, bn1_scale, bn1_shift, bn1_mean, pad, y1_origin, y1_size,
      y1_bound=None):
    _eager_only("split_head", y1_bound=y1_bound)
    b, _, d, h, w, _ = scv.shape
    return (scv.new_empty((b, 8, d, h, w), dtype=_F32), scv.new_empty([b] + list(y1_size) + [16], dtype=_F32))


@torch.library.custom_op("mvs::cost_volume_c4_bf16", mutates_args=())
def cost_volume_c4_bf16(feat: torch.Tensor, K: torch.Tensor, R: torch.Tensor, T: torch.Tensor,
                        d_min: torch.Tensor, d_int: torch.Tensor, batch_size: int, n_views: int,
                        d_begin: int, d_count: int, d_scale: float) -> torch.Tensor:
    """mvs::cost_volume_c4 stored in bf16 (SURVEY.md §8 f3 reduced-precision opt-in): the same
    layout [B, C/4, d_count, h, w, 4], each value the fp32 variance rounded to nearest-even (equal to
    cost_volume_c4(...).to(torch.bfloat16)); half the HBM write, and conv3d_k3 / conv3d_region (S2)
    read it widened to fp32.  Inference only, 2 <= n_views <= 8, C % 4 == 0."""
    _require_gpu(feat, "feature_maps")
    lib = _lib.load()
    feat = feat.to(_F32).contiguous()
    K, R, T, d_min, d_int = _cams(K, R, T, d_min, d_int, feat.device, batch_size)
    _check_geometry(feat, K, batch_size, n_views)
    n, c, h, w = feat.shape
    if c % 4:
        raise ValueError("the channel-quad cost volume needs C % 4 == 0, got C=%d" % c)
    cv = torch.empty((batch_size, c // 4, d_count, h, w, 4), device=feat.device, dtype=torch.bfloat16)
    ws = torch.empty((_ws_floats(batch_size, n_views, c, h, w, d_count),), device=feat.device,
                     dtype=_F32)
    evs = (None, None)
    if KERNEL_EVENT_HOOK is not None:
        evs = tuple(ctypes.c_void_p(e.cuda_event) for e in KERNEL_EVENT_HOOK("cost_volume"))
    st = lib.mvs_cost_volume_fwd_c4_bf16(_lib.ptr(feat), _lib.ptr(K), _lib.ptr(R), _lib.ptr(T),
                                         _lib.ptr(d_min), _lib.ptr(d_int), batch_size, n_views, c, h, w,
                                         d_begin, d_count, float(d_scale), _lib.ptr(ws), _lib.ptr(cv),
                                         _lib.stream_handle(feat.device), *evs)
    _lib.check(st, "mvs_cost_volume_fwd_c4_bf16")
    return cv


@cost_volume_c4_bf16.register_fake
def _(feat, K, R, T, d_min, d_int, batch_size, n_views, d_begin, d_count, d_scale):
    n, c, h, w = feat.shape
    return feat.new_empty((batch_size, c // 4, d_count, h, w, 4), dtype=torch.bfloat16)


@torch.library.custom_op("mvs::cost_volume_backward", mutates_args=())
def cost_volume_backward(feat: torch.Tensor, workspace: torch.Tensor, grad_cv: torch.Tensor,
                         batch_size: int, n_views: int, d_count: int,
                         deterministic: bool = False) -> torch.Tensor:
    """d <cv, grad_cv> / d feat.  ``workspace`` is the forward's (sampling matrices, packed
    features, resampled references).  ``deterministic``: 64-bit fixed-point accumulation,
    bit-identical across runs (autograd passes torch.are_deterministic_algorithms_enabled())."""
    _require_gpu(feat, "feature_maps")
    lib = _lib.load()
    feat = feat.to(_F32).contiguous()
    grad_cv = grad_cv.to(_F32).contiguous()
    n, c, h, w = feat.shape
    grad_feat = torch.empty_like(feat)
    flags = _lib.MVS_BWD_DETERMINISTIC if deterministic else 0
    nb = lib.mvs_cost_volume_bwd_workspace_bytes(batch_size, n_views, c, h, w, d_count, flags)
    bws = torch.empty((max(nb, 8) + 7) // 8, device=feat.device, dtype=torch.int64)
    st = lib.mvs_cost_volume_bwd(_lib.ptr(feat), _lib.ptr(workspace), _lib.ptr(grad_cv),
                                 batch_size, n_views, c, h, w, d_count, flags, _lib.ptr(bws),
                                 _lib.ptr(grad_feat), _lib.stream_handle(feat.device))
    _lib.check(st, "mvs_cost_volume_bwd")
    return grad_feat


@cost_volume_backward.register_fake
def _(feat, workspace, grad_cv, batch_size, n_views, d_count, deterministic=False):
    return torch.empty_like(feat)


def _cv_setup(ctx, inputs, output):
    feat, _, _, _, _, _, batch_size, n_views, _, d_count, _ = inputs
    _, ws = output
    ctx.save_for_backward(feat, ws)
    ctx.dims = (batch_size, n_views, d_count)


def _cv_backward(ctx, grad_cv, _grad_ws):
    feat, ws = ctx.saved_tensors
    batch_size, n_views, d_count = ctx.dims
    grad_feat = None
    if ctx.needs_input_grad[0] and grad_cv is not None:
        grad_feat = cost_volume_backward(feat, ws, grad_cv, batch_size, n_views, d_count,
                                         torch.are_deterministic_algorithms_enabled())
    return grad_feat, None, None, None, None, None, None, None, None, None, None


torch.library.register_autograd("mvs::cost_volume", _cv_backward, setup_context=_cv_setup)
# bf16 cost volume: the rounding is passed straight through (d round(x) / dx := 1); the fp32
# gradient kernel is reused on the upcast bf16 gradient
torch.library.register_autograd("mvs::cost_volume_bf16", _cv_backward, setup_context=_cv_setup)


# ----------------------------------------------------------------------------------------------
# mvs::homography_warp (materialised warped volume, API compatibility)
# ----------------------------------------------------------------------------------------------
@torch.library.custom_op("mvs::homography_warp", mutates_args=())
def homography_warp(feat: torch.Tensor, K: torch.Tensor, R: torch.Tensor, T: torch.Tensor,
                    d_min: torch.Tensor, d_int: torch.Tensor, batch_size: int, n_views: int,
                    d_begin: int, d_count: int, d_scale: float) -> torch.Tensor:
    """warped [B*V, C, d_count, h, w] (homography.py:6-92 output layout)."""
    _require_gpu(feat, "feature_maps")
    lib = _lib.load()
    feat = feat.to(_F32).contiguous()
    K, R, T, d_min, d_int = _cams(K, R, T, d_min, d_int, feat.device, batch_size)
    _check_geometry(feat, K, batch_size, n_views)
    n, c, h, w = feat.shape
    warped = torch.empty((n, c, d_count, h, w), device=feat.device, dtype=_F32)
    ws = torch.empty((n * d_count * 9,), device=feat.device, dtype=_F32)
    st = lib.mvs_homography_warp_fwd(_lib.ptr(feat), _lib.ptr(K), _lib.ptr(R), _lib.ptr(T),
                                     _lib.ptr(d_min), _lib.ptr(d_int), batch_size, n_views, c, h,
                                     w, d_begin, d_count, float(d_scale), _lib.ptr(ws),
                                     _lib.ptr(warped), _lib.stream_handle(feat.device))
    _lib.check(st, "mvs_homography_warp_fwd")
    return warped


@homography_warp.register_fake
def _(feat, K, R, T, d_min, d_int, batch_size, n_views, d_begin, d_count, d_scale):
    n, c, h, w = feat.shape
    return feat.new_empty((n, c, d_count, h, w))


# ----------------------------------------------------------------------------------------------
# mvs::assemble_cost_volume
# ----------------------------------------------------------------------------------------------
@torch.library.custom_op("mvs::assemble_cost_volume", mutates_args=())
def assemble_cost_volume_op(warped: torch.Tensor, n_views: int) -> torch.Tensor:
    _require_gpu(warped, "warped_feature_maps")
    lib = _lib.load()
    warped = warped.to(_F32).contiguous()
    bn, c, d, h, w = warped.shape
    if bn % n_views:
        raise ValueError("%d warped images is not a multiple of n_views=%d" % (bn, n_views))
    b = bn // n_views
    cv = torch.empty((b, c, d, h, w), device=warped.device, dtype=_F32)
    st = lib.mvs_assemble_cost_volume_fwd(_lib.ptr(warped), b, n_views, c, d, h, w, _lib.ptr(cv),
                                          _lib.stream_handle(warped.device))
    _lib.check(st, "mvs_assemble_cost_volume_fwd")
    return cv


@assemble_cost_volume_op.register_fake
def _(warped, n_views):
    bn, c, d, h, w = warped.shape
    return warped.new_empty((bn // n_views, c, d, h, w))


def _acv_setup(ctx, inputs, output):
    warped, n_views = inputs
    ctx.save_for_backward(warped)
    ctx.n_views = n_views


def _acv_backward(ctx, grad_cv):
    # d cv / d x_v = 2 (x_v - mean) / V  (costvolume.py:14); plain torch on the device
    (warped,) = ctx.saved_tensors
    v = ctx.n_views
    bn = warped.shape[0]
    x = warped.reshape((bn // v, v) + tuple(warped.shape[1:]))
    mean = x.mean(1, keepdim=True)
    g = (2.0 / v) * (x - mean) * grad_cv.unsqueeze(1)
    return g.reshape(warped.shape), None


torch.library.register_autograd("mvs::assemble_cost_volume", _acv_backward, setup_context=_acv_setup)


# ----------------------------------------------------------------------------------------------
# mvs::extract_depth_map
# ----------------------------------------------------------------------------------------------
@torch.library.custom_op("mvs::extract_depth_map", mutates_args=())
def extract_depth_map_op(prob_volume: torch.Tensor, d_batch: torch.Tensor, n_est: int) -> torch.Tensor:
    _require_gpu(prob_volume, "prob_volume")
    lib = _lib.load()
    prob = prob_volume.to(_F32).contiguous()
    if prob.dim() != 5 or prob.shape[1] != 1:
        raise ValueError("prob_volume must be [B, 1, D, h, w], got %s" % (tuple(prob.shape),))
    b, _, d, h, w = prob.shape
    db = d_batch.to(device=prob.device, dtype=_F32).reshape(-1, d)
    if db.shape[0] == 1 and b > 1:
        db = db.expand(b, d)
    db = db.contiguous()
    depth = torch.empty((b, 1, h, w), device=prob.device, dtype=_F32)
    st = lib.mvs_extract_depth_map_fwd(_lib.ptr(prob), _lib.ptr(db), b, d, h, w, int(n_est),
                                       _lib.ptr(depth), _lib.stream_handle(prob.device))
    _lib.check(st, "mvs_extract_depth_map_fwd")
    return depth


@extract_depth_map_op.register_fake
def _(prob_volume, d_batch, n_est):
    b, _, d, h, w = prob_volume.shape
    return prob_volume.new_empty((b, 1, h, w))


def _sam_setup(ctx, inputs, output):
    prob, d_batch, n_est = inputs
    ctx.save_for_backward(prob, d_batch, output)
    ctx.n_est = n_est


def _sam_backward(ctx, grad_depth):
    # depth = sum_{r in S} d_r P_r / sum_{r in S} P_r  ->  d depth / d P_r = (d_r - depth) / den
    # on S = {rank_j : j < n_est} (the mask is piecewise constant in P).  Plain torch on device.
    prob, d_batch, depth = ctx.saved_tensors
    b, _, d, h, w = prob.shape
    n_est = min(ctx.n_est, d)
    p = prob[:, 0]                                              # [B, D, h, w]
    pj = p[:, :n_est].unsqueeze(2)                              # [B, E, 1, h, w]
    idx = torch.arange(d, device=p.device)
    before = (idx.view(1, 1, d, 1, 1) < torch.arange(n_est, device=p.device).view(1, n_est, 1, 1, 1))
    rank = ((p.unsqueeze(1) > pj) | ((p.unsqueeze(1) == pj) & before)).sum(2)   # [B, E, h, w]
    mask = torch.zeros_like(p).scatter_(1, rank, 1.0)
    db = d_batch.to(p).reshape(-1, d)
    if db.shape[0] == 1 and b > 1:
        db = db.expand(b, d)
    den = (p * mask).sum(1, keepdim=True)
    g = mask * (db.view(b, d, 1, 1) - depth) / den * grad_depth
    return g.unsqueeze(1), None, None


torch.library.register_autograd("mvs::extract_depth_map", _sam_backward, setup_context=_sam_setup)


# ----------------------------------------------------------------------------------------------
# mvs::conv3d_k3 -- CostVolumeReg.conv_0_0 (32 -> 8) / conv_out (8 -> 1), model.py:77,96
# ----------------------------------------------------------------------------------------------
@torch.library.custom_op("mvs::conv3d_k3", mutates_args=())
def conv3d_k3(x: torch.Tensor, weight: torch.Tensor, bn_scale: Optional[torch.Tensor] = None,
              bn_shift: Optional[torch.Tensor] = None, bn_mean: Optional[torch.Tensor] = None,
              in_c4: bool = False, wino_z: bool = False, x2: Optional[torch.Tensor] = None,
              in_bn: Optional[torch.Tensor] = None) -> torch.Tensor:
    """nn.Conv3d(c_in, c_out, 3, stride=1, padding=1, bias=False) forward, c_out in {1, 8}, fp32
    NCDHW, on the HIP kernel (csrc/conv3d_narrow.hip); with bn_* given, max((y - mean) * scale +
    shift, 0) is fused (eval BN + ReLU).  ``in_c4``: x is the channel-quad [B, Cin/4, D, H, W, 4]
    of cost_volume_c4 (fp32) or cost_volume_c4_bf16 (bf16: widened on load, fp32 arithmetic).
    ``wino_z`` (c_out = 8): Winograd F(2,3) along depth (MVS_CONV_WINO_Z; the
    transformed weights are formed in float64 here).  ``x2`` + ``in_bn`` (c_out 1, NCDHW): the input is
    relu(BN_a(x)) + relu(BN_b(x2)) per channel, in_bn fp32 [6, c_in] (train mode's conv_out input,
    formed on load).  Inference only (no autograd formula): CostVolumeReg uses it on the no-grad path."""
    _require_gpu(x, "x")
    lib = _lib.load()
    if in_c4:
        if x.dim() != 6 or x.shape[-1] != 4:
            raise ValueError("in_c4: x [B, Cin/4, D, H, W, 4] expected, got %s" % (tuple(x.shape),))
        b, c4, d, h, wd, _ = x.shape
        cin = 4 * c4
    else:
        if x.dim() != 5:
            raise ValueError("x [B, Cin, D, H, W] expected, got %s" % (tuple(x.shape),))
        b, cin, d, h, wd = x.shape
    if weight.dim() != 5 or tuple(weight.shape[2:]) != (3, 3, 3) or weight.shape[1] != cin:
        raise ValueError("weight [Cout, %d, 3, 3, 3] expected, got %s" % (cin, tuple(weight.shape)))
    quad_bf16 = in_c4 and x.dtype == torch.bfloat16
    x = x.contiguous() if quad_bf16 else x.to(_F32).contiguous()
    cout = weight.shape[0]
    # the kernel reads weight[c_in][3][3][3][c_out] (pairs of output channels per 8-byte load)
    if wino_z and cout != 8:
        raise ValueError("wino_z needs c_out = 8")
    if wino_z:
        w = derived("k3wz", (weight,), lambda wt: _wino_z_weight(wt).to(device=x.device), x.device)
    else:
        w = derived("k3", (weight,), lambda wt: wt.to(device=x.device, dtype=_F32).permute(1, 2, 3, 4, 0).contiguous(),
                    x.device)
    bn = [t if t is None else t.to(device=x.device, dtype=_F32).contiguous() for t in (bn_scale, bn_shift, bn_mean)]
    if any(t is None for t in bn) and not all(t is None for t in bn):
        raise ValueError("bn_scale, bn_shift and bn_mean go together")
    bp = [None if t is None else _lib.ptr(t) for t in bn]
    y = torch.empty((b, cout, d, h, wd), device=x.device, dtype=_F32)
    flags = ((_lib.MVS_CONV_IN_C4 if in_c4 else 0) | (_lib.MVS_CONV_WINO_Z if wino_z else 0)
             | (_lib.MVS_CONV_IN_BF16 if quad_bf16 else 0))
    if (x2 is None) != (in_bn is None):
        raise ValueError("x2 and in_bn go together")
    if x2 is not None:
        if x2.shape != x.shape or in_bn.shape != (6, cin):
            raise ValueError("x2 of x's shape and in_bn [6, c_in] expected")
        x2 = x2.to(_F32).contiguous()
        in_bn = in_bn.to(device=x.device, dtype=_F32).contiguous()
    st = lib.mvs_conv3d_k3_fwd(_lib.ptr(x), flags, _lib.ptr(w), _lib.ptr(y),
                               b, cin, cout, d, h, wd, *bp, None if x2 is None else _lib.ptr(x2),
                               None if in_bn is None else _lib.ptr(in_bn), _lib.stream_handle(x.device))
    _lib.check(st, "mvs_conv3d_k3_fwd")
    return y


WGRAD_SHAPES = ((32, 8), (16, 8), (8, 8), (8, 1))   # (c_in, c_out) of mvs_conv3d_k3_wgrad


def conv3d_k3_wgrad(x: torch.Tensor, gy: torch.Tensor) -> torch.Tensor:
    """Weight gradient of nn.Conv3d(c_in, c_out, 3, padding=1, bias=False) (model.py:101 conv_0_0,
    model.py:124 conv_out) from its input x [B, c_in, D, H, W] and output gradient gy [B, c_out, D, H, W]
    (fp32 NCDHW): dw [c_out, c_in, 3, 3, 3] on the f32 matrix cores (mvs_conv3d_k3_wgrad, deterministic).
    (c_in, c_out) in WGRAD_SHAPES."""
    _require_gpu(x, "x")
    lib = _lib.load()
    if x.dim() != 5 or gy.dim() != 5 or x.shape[0] != gy.shape[0] or x.shape[2:] != gy.shape[2:]:
        raise ValueError("x [B, c_in, D, H, W] and gy [B, c_out, D, H, W] expected")
    b, cin, d, h, w = x.shape
    cout = gy.shape[1]
    if (cin, cout) not in WGRAD_SHAPES:
        raise ValueError("(c_in, c_out) = (%d, %d) not in %s" % (cin, cout, WGRAD_SHAPES))
    x = x.to(_F32).contiguous()
    gy = gy.to(_F32).contiguous()
    ws = torch.empty(lib.mvs_conv3d_k3_wgrad_workspace_bytes(b, cin, d, h, w) // 4, device=x.device, dtype=_F32)
    dw = torch.empty((cout, cin, 3, 3, 3), device=x.device, dtype=_F32)
    st = lib.mvs_conv3d_k3_wgrad(_lib.ptr(x), _lib.ptr(gy), b, cin, cout, d, h, w, _lib.ptr(dw), _lib.ptr(ws),
                                 _lib.stream_handle(x.device))
    _lib.check(st, "mvs_conv3d_k3_wgrad")
    return dw


@torch.library.custom_op("mvs::conv_head_fp32", mutates_args=())
def conv_head_fp32(cv4: torch.Tensor, w0: torch.Tensor, bn0_scale: Optional[torch.Tensor],
                   bn0_shift: Optional[torch.Tensor], bn0_mean: Optional[torch.Tensor], w1: torch.Tensor,
                   bn1_scale: Optional[torch.Tensor], bn1_shift: Optional[torch.Tensor],
                   bn1_mean: Optional[torch.Tensor], pad: list[int], y1_origin: list[int],
                   y1_size: list[int]) -> tuple[torch.Tensor, torch.Tensor]:
    """conv_0_0 + BN_0 + ReLU (model.py:101, whole volume) and conv_1_0 + BN_1 + ReLU (model.py:103, on the
    region y1_origin + [0, y1_size)) of the fp32 channel-quad cost volume ``cv4`` [B, 8, D, H, W, 4]
    (cost_volume_c4) in ONE pass over it, in exact fp32 (mvs_conv_head_fp32_fwd: conv_0_0 on the VALU with
    the depth-Winograd transform, conv_1_0 on the fp32 matrix cores from the same LDS tiles).  ``w0`` /
    ``w1``: the modules' weights [8, 32, 3, 3, 3] / [16, 32, 3, 3, 3].  Returns (y0 [B, 8, D, H, W],
    y1 [B, *y1_size, 16] channels-last).  Every pad odd (config.py:20 at even dims).  Inference only."""
    _require_gpu(cv4, "cv4")
    lib = _lib.load()
    if cv4.dim() != 6 or cv4.shape[1] != 8 or cv4.shape[5] != 4 or cv4.dtype != _F32:
        raise ValueError("cv4: the fp32 channel-quad cost volume [B, 8, D, H, W, 4]")
    if tuple(w0.shape) != (8, 32, 3, 3, 3) or tuple(w1.shape) != (16, 32, 3, 3, 3):
        raise ValueError("w0 [8, 32, 3, 3, 3] and w1 [16, 32, 3, 3, 3] expected")
    cv4 = cv4.contiguous()
    dev = cv4.device
    b, _, d, h, wd, _ = cv4.shape
    w0z = derived("k3wz", (w0,), lambda wt: _wino_z_weight(wt).to(device=dev), dev)
    w1r = derived("head1_region", (w1,), lambda wt: wt.detach().to(device=dev, dtype=_F32).permute(2, 3, 4, 0, 1)
                  .reshape(27, 16, 32).contiguous(), dev)
    w1p = derived("head1_pass", (w1,), lambda wt: w1r.view(27, 16, 8, 4).permute(2, 0, 1, 3).contiguous(), dev)
    bns = []
    for t in (bn0_scale, bn0_shift, bn0_mean, bn1_scale, bn1_shift, bn1_mean):
        bns.append(None if t is None else t.to(device=dev, dtype=_F32).contiguous())
    y0 = torch.empty((b, 8, d, h, wd), device=dev, dtype=_F32)
    y1 = torch.empty([b] + [int(v) for v in y1_size] + [16], device=dev, dtype=_F32)
    bp = [None if t is None else _lib.ptr(t) for t in bns]
    evs = (None, None)
    if KERNEL_EVENT_HOOK is not None:   # around the fused kernel (bench.py's fp32 roofline kernel)
        evs = tuple(ctypes.c_void_p(e.cuda_event) for e in KERNEL_EVENT_HOOK("conv_head"))
    st = lib.mvs_conv_head_fp32_fwd(_lib.ptr(cv4), b, d, h, wd, _lib.ptr(w0z), *bp[:3], _lib.ptr(w1r), _lib.ptr(w1p),
                                    *bp[3:], _ints3(pad), _ints3(y1_origin), _ints3(y1_size), _lib.ptr(y0), _lib.ptr(y1),
                                    _lib.stream_handle(dev), *evs)
    _lib.check(st, "mvs_conv_head_fp32_fwd")
    return y0, y1


@conv_head_fp32.register_fake
def _(cv4, w0, bn0_scale, bn0_shift, bn0_mean, w1, bn1_scale, bn1_shift, bn1_mean, pad, y1_origin, y1_size):
    b, _, d, h, w, _ = cv4.shape
    return (cv4.new_empty((b, 8, d, h, w), dtype=_F32),
            cv4.new_empty([b] + [int(v) for v in y1_size] + [16], dtype=_F32))


@torch.library.custom_op("mvs::conv3d_k3_split", mutates_args=())
def conv3d_k3_split(x: torch.Tensor, absmax: Optional[torch.Tensor], weight: torch.Tensor,
                    bn_scale: Optional[torch.Tensor] = None, bn_shift: Optional[torch.Tensor] = None,
                    bn_mean: Optional[torch.Tensor] = None) -> torch.Tensor:
    """conv_0_0 (nn.Conv3d(32, 8, 3, padding=1, bias=False), + eval BN + ReLU when bn_* are given)
    over the channel-quad fp32 cost volume x [B, 8, D, H, W, 4] on the f16 matrix cores with split
    operands (csrc/conv3d_split.hip, mvs_conv3d_k3_split_fwd): fp32-level error, not bit-equal to
    conv3d_k3.  ``absmax``: the volume's bound words (cost_volume_c4_absmax); None = unscaled (every
    |x| < 2^15 must hold).  Inference only."""
    _require_gpu(x, "x")
    lib = _lib.load()
    if x.dim() != 6 or tuple(x.shape[1:2]) + tuple(x.shape[-1:]) != (8, 4) or x.dtype not in (_F32, torch.int32):
        raise ValueError("x: fp32 or split (int32) channel-quad [B, 8, D, H, W, 4] expected, got %s %s"
                         % (tuple(x.shape), x.dtype))
    split_in = x.dtype == torch.int32
    if split_in and absmax is None:
        raise ValueError("the split cost volume needs its bound words (absmax)")
    if tuple(weight.shape) != (8, 32, 3, 3, 3):
        raise ValueError("weight [8, 32, 3, 3, 3] expected, got %s" % (tuple(weight.shape),))
    x = x.contiguous()
    b, _, d, h, wd, _ = x.shape
    frag, wexp = derived("k3split", (weight,), lambda wt: split_weight_fragments(wt, x.device), x.device)
    bn = [t if t is None else t.to(device=x.device, dtype=_F32).contiguous() for t in (bn_scale, bn_shift, bn_mean)]
    if any(t is None for t in bn) and not all(t is None for t in bn):
        raise ValueError("bn_scale, bn_shift and bn_mean go together")
    bp = [None if t is None else _lib.ptr(t) for t in bn]
    if absmax is not None:
        if absmax.numel() != 8 or absmax.dtype != torch.int32 or absmax.device != x.device:
            raise ValueError("absmax: int32[8] on the volume's device expected")
        absmax = absmax.contiguous()
    y = torch.empty((b, 8, d, h, wd), device=x.device, dtype=_F32)
    st = lib.mvs_conv3d_k3_split_fwd(_lib.ptr(x), _lib.MVS_CONV_IN_SPLIT if split_in else 0, _lib.ptr(frag), int(wexp),
                                     None if absmax is None else _lib.ptr(absmax), _lib.ptr(y),
                                     b, d, h, wd, *bp, _lib.stream_handle(x.device))
    _lib.check(st, "mvs_conv3d_k3_split_fwd")
    return y


@conv3d_k3_split.register_fake
def _(x, absmax, weight, bn_scale=None, bn_shift=None, bn_mean=None):
    return x.new_empty((x.shape[0], 8) + tuple(x.shape[2:5]), dtype=_F32)


@torch.library.custom_op("mvs::conv_s2_split", mutates_args=())
def conv_s2_split(x: torch.Tensor, absmax: Optional[torch.Tensor], weight: torch.Tensor, dims: list[int],
                  out_origin: list[int], out_size: list[int], pad: list[int], bn_scale: Optional[torch.Tensor] = None,
                  bn_shift: Optional[torch.Tensor] = None, bn_mean: Optional[torch.Tensor] = None) -> torch.Tensor:
    """conv_1_0 (nn.Conv3d(32, 16, 3, stride=2, padding=pad, bias=False), + eval BN + ReLU when bn_*
    are given) of the channel-quad fp32 cost volume x [B, 8, D, H, W, 4] on the output region
    [out_origin, out_origin + out_size), split-fp16 MFMA (csrc/conv3d_s2_split.hip,
    mvs_conv3d_s2_split_fwd) -> channels-last region [B, out_size..., 16] (conv3d_region's S2 layout).
    ``absmax``: the volume's bound words (cost_volume_c4_absmax), None = unscaled.  Inference only."""
    _require_gpu(x, "x")
    lib = _lib.load()
    if x.dim() != 6 or x.shape[1] != 8 or x.shape[-1] != 4 or x.dtype not in (_F32, torch.int32):
        raise ValueError("x: fp32 or split (int32) channel-quad [B, 8, D, H, W, 4] expected, got %s %s"
                         % (tuple(x.shape), x.dtype))
    split_in = x.dtype == torch.int32
    if split_in and absmax is None:
        raise ValueError("the split cost volume needs its bound words (absmax)")
    if tuple(weight.shape) != (16, 32, 3, 3, 3):
        raise ValueError("weight [16, 32, 3, 3, 3] expected, got %s" % (tuple(weight.shape),))
    if list(x.shape[2:5]) != [int(v) for v in dims]:
        raise ValueError("dims %s do not match the volume %s" % (list(dims), list(x.shape[2:5])))
    x = x.contiguous()
    frag, wexp = derived("s2split", (weight,), lambda wt: _s2_split_fragments(wt, x.device), x.device)
    bn = [t if t is None else t.to(device=x.device, dtype=_F32).contiguous() for t in (bn_scale, bn_shift, bn_mean)]
    if any(t is None for t in bn) and not all(t is None for t in bn):
        raise ValueError("bn_scale, bn_shift and bn_mean go together")
    bp = [None if t is None else _lib.ptr(t) for t in bn]
    if absmax is not None:
        if absmax.numel() != 8 or absmax.dtype != torch.int32 or absmax.device != x.device:
            raise ValueError("absmax: int32[8] on the volume's device expected")
        absmax = absmax.contiguous()
    y = torch.empty([x.shape[0]] + [int(v) for v in out_size] + [16], device=x.device, dtype=_F32)
    st = lib.mvs_conv3d_s2_split_fwd(_lib.ptr(x), _lib.MVS_CONV_IN_SPLIT if split_in else 0, _lib.ptr(frag), int(wexp),
                                     None if absmax is None else _lib.ptr(absmax), _lib.ptr(y), x.shape[0],
                                     _ints3(dims), _ints3(out_origin), _ints3(out_size), _ints3(pad), *bp,
                                     _lib.stream_handle(x.device))
    _lib.check(st, "mvs_conv3d_s2_split_fwd")
    return y


@conv_s2_split.register_fake
def _(x, absmax, weight, dims, out_origin, out_size, pad, bn_scale=None, bn_shift=None, bn_mean=None):
    return x.new_empty([x.shape[0]] + [int(v) for v in out_size] + [16], dtype=_F32)


def _s2_split_fragments(weight, device):
    lib = _lib.load()
    w = weight.detach().to(device="cpu", dtype=_F32).contiguous()
    frag = torch.empty((27 * 2 * 64 * 8,), dtype=torch.int16)
    e = ctypes.c_int(0)
    st = lib.mvs_conv3d_s2_split_weights(_lib.ptr(w), _lib.ptr(frag), ctypes.byref(e))
    _lib.check(st, "mvs_conv3d_s2_split_weights")
    return frag.to(device), e.value


def split_weight_fragments(weight, device):
    """(fp16 MFMA fragments [27*64*8] int16 on ``device``, exponent) of conv_0_0's weight, formed on
    the host by mvs_conv3d_split_weights (the C ABI's own split, so every caller gets the same)."""
    lib = _lib.load()
    w = weight.detach().to(device="cpu", dtype=_F32).contiguous()
    frag = torch.empty((27 * 64 * 8,), dtype=torch.int16)
    e = ctypes.c_int(0)
    st = lib.mvs_conv3d_split_weights(_lib.ptr(w), _lib.ptr(frag), ctypes.byref(e))
    _lib.check(st, "mvs_conv3d_split_weights")
    return frag.to(device), e.value


def _wino_z_weight(wt):
    """Conv3d weight [co][ci][kd][ky][kx] -> the depth-Winograd F(2,3) weight wu[ci][ky][kx][4][co]:
    per depth column g0..g2 the transformed taps (g0, (g0 + g1 + g2) / 2, (g0 - g1 + g2) / 2, g2),
    formed in float64 and rounded once (csrc/conv3d_narrow.hip, WZ)."""
    g = wt.detach().double()
    g0, g1, g2 = g[:, :, 0], g[:, :, 1], g[:, :, 2]
    u = torch.stack((g0, (g0 + g1 + g2) * 0.5, (g0 - g1 + g2) * 0.5, g2), dim=2)   # [co][ci][4][ky][kx]
    return u.permute(1, 3, 4, 2, 0).contiguous().to(_F32)


@conv3d_k3.register_fake
def _(x, weight, bn_scale=None, bn_shift=None, bn_mean=None, in_c4=False, wino_z=False, x2=None, in_bn=None):
    return x.new_empty((x.shape[0], weight.shape[0]) + tuple(x.shape[2:5]))


# ----------------------------------------------------------------------------------------------
# mvs::conv2d -- FeatureEncoder / refinement Conv2d (+ eval BatchNorm2d + ReLU), model.py:22-65,134-145
# ----------------------------------------------------------------------------------------------
# (c_in, c_out, k, stride) with a kernel instantiation (csrc/conv2d_narrow.hip)
CONV2D_SHAPES = frozenset({(3, 8, 3, 1), (8, 8, 3, 1), (8, 16, 5, 2), (16, 16, 3, 1), (16, 32, 5, 2),
                           (32, 32, 3, 1), (4, 32, 3, 1), (32, 1, 3, 1)})


def conv2d_supported(conv):
    """nn.Conv2d the HIP kernel runs: bias-free, padding k/2, no dilation/groups, a listed shape."""
    k = conv.kernel_size[0]
    return (conv.bias is None and conv.kernel_size == (k, k) and conv.stride[0] == conv.stride[1]
            and conv.padding == (k // 2, k // 2) and conv.dilation == (1, 1) and conv.groups == 1
            and conv.padding_mode == "zeros"
            and (conv.in_channels, conv.out_channels, k, conv.stride[0]) in CONV2D_SHAPES)


# (y_bound is raised in place; not declared as a mutation, as conv3d_region_split's bound words)
@torch.library.custom_op("mvs::conv2d", mutates_args=())
def conv2d(x: torch.Tensor, weight: torch.Tensor, stride: int, bn_scale: Optional[torch.Tensor] = None,
           bn_shift: Optional[torch.Tensor] = None, bn_mean: Optional[torch.Tensor] = None,
           y_bound: Optional[torch.Tensor] = None) -> torch.Tensor:
    """nn.Conv2d(c_in, c_out, k, stride, padding=k // 2, bias=False) forward, fp32 NCHW, on the HIP
    kernel (csrc/conv2d_narrow.hip); with bn_* given, max((y - mean) * scale + shift, 0) is fused
    (eval BatchNorm2d + ReLU).  ``y_bound``: None or zeroed bound words (bound_words) raised to
    max|y|, the input scale of a following conv2d_split.  Shapes: CONV2D_SHAPES.  Inference only (no
    autograd formula)."""
    _require_gpu(x, "x")
    lib = _lib.load()
    if x.dim() != 4 or weight.dim() != 4 or weight.shape[1] != x.shape[1] or weight.shape[2] != weight.shape[3]:
        raise ValueError("x [N, C, H, W] and weight [Cout, C, k, k] expected, got %s, %s"
                         % (tuple(x.shape), tuple(weight.shape)))
    n, cin, h, wd = x.shape
    cout, k = weight.shape[0], weight.shape[2]
    x = x.to(_F32).contiguous()
    # the kernel reads weight[c_in][k][k][c_out] (pairs of output channels per 8-byte scalar load)
    w = derived("conv2d", (weight,), lambda wt: wt.to(device=x.device, dtype=_F32).permute(1, 2, 3, 0).contiguous(),
                x.device)
    bn = [t if t is None else t.to(device=x.device, dtype=_F32).contiguous() for t in (bn_scale, bn_shift, bn_mean)]
    if any(t is None for t in bn) and not all(t is None for t in bn):
        raise ValueError("bn_scale, bn_shift and bn_mean go together")
    bp = [None if t is None else _lib.ptr(t) for t in bn]
    ho, wo = (h + 2 * (k // 2) - k) // stride + 1, (wd + 2 * (k // 2) - k) // stride + 1
    y = torch.empty((n, cout, ho, wo), device=x.device, dtype=_F32)
    st = lib.mvs_conv2d_fwd(_lib.ptr(x), _lib.ptr(w), _lib.ptr(y), n, cin, cout, h, wd, k, stride, *bp,
                            _bound_ptr(y_bound), _lib.stream_handle(x.device))
    _lib.check(st, "mvs_conv2d_fwd")
    return y


@conv2d.register_fake
def _(x, weight, stride, bn_scale=None, bn_shift=None, bn_mean=None, y_bound=None):
    _eager_only("conv2d", y_bound=y_bound)
    k = weight.shape[2]
    return x.new_empty((x.shape[0], weight.shape[0], (x.shape[2] + 2 * (k // 2) - k) // stride + 1,
                        (x.shape[3] + 2 * (k // 2) - k) // stride + 1))


# (c_in, c_out, k, stride) of the split-fp16 MFMA kernel (csrc/conv2d_split.hip): the encoder's layers
# 2-8 and the refinement net's 32 -> 32
CONV2D_SPLIT_SHAPES = frozenset({(8, 8, 3, 1), (8, 16, 5, 2), (16, 16, 3, 1), (16, 32, 5, 2), (32, 32, 3, 1)})


def conv2d_split_fragments(weight, device):
    """(split-fp16 MFMA fragments on ``device``, exponent) of an nn.Conv2d weight [c_out][c_in][k][k],
    formed on the host by mvs_conv2d_split_weights."""
    lib = _lib.load()
    w = weight.detach().to(device="cpu", dtype=_F32).contiguous()
    cout, cin, k, _ = w.shape
    kb = -(-(k * k) // (32 // cin))
    parts = 1 if cout == 8 else 2 * (cout // 16)
    frag = torch.empty((kb * parts * 64 * 8,), dtype=torch.int16)
    e = ctypes.c_int(0)
    st = lib.mvs_conv2d_split_weights(_lib.ptr(w), cin, cout, k, _lib.ptr(frag), ctypes.byref(e))
    _lib.check(st, "mvs_conv2d_split_weights")
    return frag.to(device), e.value


# (y_bound is raised in place; not declared as a mutation, as conv3d_region_split's bound words)
@torch.library.custom_op("mvs::conv2d_split", mutates_args=())
def conv2d_split(x: torch.Tensor, weight: torch.Tensor, stride: int, x_bound: torch.Tensor,
                 y_bound: Optional[torch.Tensor] = None, bn_scale: Optional[torch.Tensor] = None,
                 bn_shift: Optional[torch.Tensor] = None, bn_mean: Optional[torch.Tensor] = None) -> torch.Tensor:
    """conv2d on the f16 matrix cores with split operands (mvs_conv2d_split_fwd,
    csrc/conv2d_split.hip): x scaled by its bound words ``x_bound`` (raised by the conv2d /
    conv2d_split that produced x), ``y_bound`` (None or zeroed words) raised to max|y|.  Same
    arguments and epilogue as conv2d otherwise; fp32-level error, not conv2d's bit pattern.  Shapes:
    CONV2D_SPLIT_SHAPES.  Inference only."""
    _require_gpu(x, "x")
    lib = _lib.load()
    if x.dim() != 4 or weight.dim() != 4 or weight.shape[1] != x.shape[1] or weight.shape[2] != weight.shape[3]:
        raise ValueError("x [N, C, H, W] and weight [Cout, C, k, k] expected, got %s, %s"
                         % (tuple(x.shape), tuple(weight.shape)))
    n, cin, h, wd = x.shape
    cout, k = weight.shape[0], weight.shape[2]
    if (cin, cout, k, stride) not in CONV2D_SPLIT_SHAPES:
        raise ValueError("conv2d_split: unsupported (c_in, c_out, k, stride) %s" % ((cin, cout, k, stride),))
    x = x.to(_F32).contiguous()
    dev = x.device
    frag, ew = derived("conv2d_split", (weight,), lambda wt: conv2d_split_fragments(wt, dev), dev)
    bn = [t if t is None else t.to(device=dev, dtype=_F32).contiguous() for t in (bn_scale, bn_shift, bn_mean)]
    if any(t is None for t in bn) and not all(t is None for t in bn):
        raise ValueError("bn_scale, bn_shift and bn_mean go together")
    bp = [None if t is None else _lib.ptr(t) for t in bn]
    ho, wo = (h + 2 * (k // 2) - k) // stride + 1, (wd + 2 * (k // 2) - k) // stride + 1
    y = torch.empty((n, cout, ho, wo), device=dev, dtype=_F32)
    st = lib.mvs_conv2d_split_fwd(_lib.ptr(x), _lib.ptr(frag), ew, _lib.ptr(y), n, cin, cout, h, wd, k, stride,
                                  *bp, _bound_ptr(x_bound), _bound_ptr(y_bound), _lib.stream_handle(dev))
    _lib.check(st, "mvs_conv2d_split_fwd")
    return y


@conv2d_split.register_fake
def _(x, weight, stride, x_bound, y_bound=None, bn_scale=None, bn_shift=None, bn_mean=None):
    _eager_only("conv2d_split", y_bound=y_bound)
    k = weight.shape[2]
    return x.new_empty((x.shape[0], weight.shape[0], (x.shape[2] + 2 * (k // 2) - k) // stride + 1,
                        (x.shape[3] + 2 * (k // 2) - k) // stride + 1))


# ----------------------------------------------------------------------------------------------
# mvs::deconv3d_k3s2 -- CostVolumeReg.deconv_1_0 + BN_0 + ReLU + `+ y0` (model.py:121-123)
# ----------------------------------------------------------------------------------------------
@torch.library.custom_op("mvs::deconv3d_k3s2", mutates_args=())
def deconv3d_k3s2(x: torch.Tensor, origin: list[int], weight: torch.Tensor, out_dims: list[int],
                  pad: list[int], bn_scale: Optional[torch.Tensor], bn_shift: Optional[torch.Tensor],
                  bn_mean: Optional[torch.Tensor], residual: Optional[torch.Tensor],
                  x2: Optional[torch.Tensor] = None, channels_last: bool = False) -> torch.Tensor:
    """ConvTranspose3d(c_in, 8, 3, stride 2, padding pad) of the region tensor x (+ x2) (input region
    starting at `origin`; [B, c_in, r...] or, channels_last, [B, r..., c_in]) into the full volume
    out_dims, then max((y - mean) * scale + shift, 0) + residual (csrc/deconv3d_region.hip); without
    bn_* the raw transposed conv (+ residual if given).  Inference only."""
    _require_gpu(x, "x")
    lib = _lib.load()
    x = x.to(_F32).contiguous()
    if channels_last:
        b, rd, rh, rw, cin = x.shape
    else:
        b, cin, rd, rh, rw = x.shape
    if x2 is not None:
        x2 = x2.to(_F32).contiguous()
        if x2.shape != x.shape:
            raise ValueError("x2 must have x's shape")
    if tuple(weight.shape) != (cin, 8, 3, 3, 3):
        raise ValueError("weight [c_in, 8, 3, 3, 3] expected, got %s" % (tuple(weight.shape),))
    # tap-major weight[c_in][27][8]: the packed-FMA form (either input layout)
    w = derived("deconv_taps", (weight,),
                lambda wt: wt.to(device=x.device, dtype=_F32).reshape(cin, 8, 27).transpose(1, 2).contiguous(),
                x.device)
    flags = _lib.MVS_DECONV_WEIGHT_TAPS | (_lib.MVS_LAYOUT_CHANNELS_LAST if channels_last else 0)
    d, h, wd = out_dims
    f = lambda t: None if t is None else t.to(device=x.device, dtype=_F32).contiguous()
    sc, sh, mu, res = f(bn_scale), f(bn_shift), f(bn_mean), f(residual)
    if (sc is None) != (sh is None) or (sc is None) != (mu is None):
        raise ValueError("bn_scale, bn_shift and bn_mean go together")
    if res is not None and tuple(res.shape) != (b, 8, d, h, wd):
        raise ValueError("residual must be [B, 8, D, H, W]")
    y = torch.empty((b, 8, d, h, wd), device=x.device, dtype=_F32)
    pt = lambda t: None if t is None else _lib.ptr(t)
    st = lib.mvs_deconv3d_k3s2_fwd(_lib.ptr(x), pt(x2), flags, b, cin, 8, rd, rh,
                                   rw, *origin, _lib.ptr(w), d, h, wd, *pad, pt(sc), pt(sh), pt(mu), pt(res),
                                   _lib.ptr(y), _lib.stream_handle(x.device))
    _lib.check(st, "mvs_deconv3d_k3s2_fwd")
    return y


@deconv3d_k3s2.register_fake
def _(x, origin, weight, out_dims, pad, bn_scale, bn_shift, bn_mean, residual, x2=None, channels_last=False):
    return x.new_empty((x.shape[0], 8) + tuple(out_dims))


# ----------------------------------------------------------------------------------------------
# mvs::conv3d_region -- the regulariser's region convolutions on the fp32 MFMA (model.py:101-121)
# ----------------------------------------------------------------------------------------------
CONV_S1, CONV_S2, CONV_T2 = _lib.MVS_CONV_S1, _lib.MVS_CONV_S2, _lib.MVS_CONV_T2


_DERIVED = {}   # (tag, id(t)...) -> (weak refs, state, out): ONE entry per (tag, tensors)


def _evict(key):
    return lambda _ref: _DERIVED.pop(key, None)


def derived(tag, tensors, fn, device=None):
    """fn(*tensors), cached for inference: a kernel-layout weight or an eval-BN scale is formed once
    per parameter state instead of by a few small device ops on every forward.

    One entry per (tag, tensor identities), holding only the LATEST state: the tensors' storage and
    in-place version counters (optimizer steps, load_state_dict and running-statistic updates all bump
    them) and the target ``device`` the result is formed for (a CPU weight used with inputs on two
    GPUs gets one result per call site's device, recomputed on a device change).  A state change
    replaces the entry, so stale results are dropped instead of accumulating; the entry dies with its
    tensors (weak-reference callbacks).  Writes through ``param.data`` do not bump the version counter
    (``.data`` is a separate autograd view); code that updates weights that way must call
    ``clear_derived()``.  Never cached while autograd records (the result must carry the graph)."""
    if torch.is_grad_enabled() and any(t.requires_grad for t in tensors):
        return fn(*tensors)
    key = (tag,) + tuple(id(t) for t in tensors)
    state = tuple((t.data_ptr(), t._version) for t in tensors) + (None if device is None else str(device),)
    hit = _DERIVED.get(key)
    if hit is not None and all(r() is t for r, t in zip(hit[0], tensors)) and hit[1] == state:
        return hit[2]
    out = fn(*tensors)
    _DERIVED[key] = ([weakref.ref(t, _evict(key)) for t in tensors], state, out)
    if _pipeline_lane() and torch.cuda.is_available():
        # formed on one lane's stream of MVSNet's sample-pipelined forward, then read on every lane's: the
        # first formation completes before any lane reads it (a cache miss only: after a weight change)
        torch.cuda.current_stream().synchronize()
    return out


def _pipeline_lane():
    from . import model
    return model._LANE[0]


def clear_derived():
    """Drop every cached derived weight (after weight writes the version counters do not see)."""
    _DERIVED.clear()


def region_weight(module):
    """weight[27][c_out][c_in] of an nn.Conv3d / nn.ConvTranspose3d (mvs_conv3d_region_fwd layout)."""
    if isinstance(module, torch.nn.ConvTranspose3d):
        return derived("region_t", (module.weight,),
                       lambda w: w.permute(2, 3, 4, 1, 0).reshape(27, w.shape[1], w.shape[0]).contiguous())
    return derived("region", (module.weight,),
                   lambda w: w.permute(2, 3, 4, 0, 1).reshape(27, w.shape[0], w.shape[1]).contiguous())


def _ints3(v):
    return (ctypes.c_int * 3)(*[int(a) for a in v])


# (the bound words are raised in place; not declared as a mutation: torch's ADInplaceOrView wrapper
# indexes every declared mutable argument positionally, which fails for an omitted trailing default)
@torch.library.custom_op("mvs::conv3d_region", mutates_args=())
def conv3d_region(x: torch.Tensor, x2: Optional[torch.Tensor], weight: torch.Tensor, mode: int,
                  dims: list[int], out_origin: list[int], out_size: list[int],
                  in_origin: Optional[list[int]], in_size: Optional[list[int]], pad: Optional[list[int]],
                  bn_scale: Optional[torch.Tensor] = None, bn_shift: Optional[torch.Tensor] = None,
                  bn_mean: Optional[torch.Tensor] = None, out_ncdhw: bool = False,
                  in_c4: bool = False, absmax: Optional[torch.Tensor] = None,
                  y_bound: Optional[torch.Tensor] = None, per_lane: bool = False,
                  s2_lds: bool = False) -> torch.Tensor:
    """Region convolution (mvs_conv3d_region_fwd): mode CONV_S2 reads the full NCDHW volume x
    (in_c4: the channel-quad [B, C/4, D, H, W, 4] of cost_volume_c4, or bf16 of cost_volume_c4_bf16;
    with in_origin / in_size, x holds only that box of the volume: the fused head's stored box),
    CONV_S1 / CONV_T2 a channels-last region tensor x (+ x2) on in_origin + [0, in_size); returns the
    channels-last region tensor [B, *out_size, c_out] ([B, c_out, *out_size] with out_ncdhw), eval
    BN + ReLU fused when bn_* are given.  ``weight`` is region_weight(module).  ``y_bound``: zeroed
    bound words (int32 [MVS_BOUND_WORDS]) raised to max|y|.  ``per_lane``: the per-lane-operand kernel
    even where an LDS-staged one applies (bit-identical; tests, A/B).  ``s2_lds``: conv_1_0's shape on the
    LDS-staged stride-2 kernel (MVS_CONV_S2_LDS; opt-in).  Inference only."""
    _require_gpu(x, "x")
    lib = _lib.load()
    quad_bf16 = in_c4 and x.dtype == torch.bfloat16
    quad_split = in_c4 and x.dtype == torch.int32   # the split cost volume (absmax: its bound words)
    if quad_split and (absmax is None or absmax.numel() != 8 or absmax.dtype != torch.int32):
        raise ValueError("the split cost volume needs its bound words (absmax, int32[8])")
    x = x.contiguous() if (quad_bf16 or quad_split) else x.to(_F32).contiguous()
    if x2 is not None:
        x2 = x2.to(_F32).contiguous()
    w = weight.to(device=x.device, dtype=_F32).contiguous()
    _, cout, cin = w.shape
    b = x.shape[0]
    bn = [t if t is None else t.to(device=x.device, dtype=_F32).contiguous() for t in (bn_scale, bn_shift, bn_mean)]
    if any(t is None for t in bn) and not all(t is None for t in bn):
        raise ValueError("bn_scale, bn_shift and bn_mean go together")
    shape = (b, cout) + tuple(out_size) if out_ncdhw else (b,) + tuple(out_size) + (cout,)
    y = torch.empty(shape, device=x.device, dtype=_F32)
    flags = ((_lib.MVS_CONV_OUT_NCDHW if out_ncdhw else 0) | (_lib.MVS_CONV_IN_C4 if in_c4 else 0)
             | (_lib.MVS_CONV_IN_BF16 if quad_bf16 else 0) | (_lib.MVS_CONV_IN_SPLIT if quad_split else 0)
             | (_lib.MVS_CONV_PER_LANE if per_lane else 0) | (_lib.MVS_CONV_S2_LDS if s2_lds else 0))
    st = lib.mvs_conv3d_region_fwd(int(mode), flags, _lib.ptr(x), None if x2 is None else _lib.ptr(x2), _lib.ptr(w),
                                   _lib.ptr(y), b, cin, cout, _ints3(dims), _ints3(out_origin), _ints3(out_size),
                                   None if in_origin is None else _ints3(in_origin),
                                   None if in_size is None else _ints3(in_size),
                                   None if pad is None else _ints3(pad),
                                   *[None if t is None else _lib.ptr(t) for t in bn],
                                   _lib.ptr(absmax.contiguous()) if quad_split else None,
                                   _bound_ptr(y_bound), _lib.stream_handle(x.device))
    _lib.check(st, "mvs_conv3d_region_fwd")
    return y


@conv3d_region.register_fake
def _(x, x2, weight, mode, dims, out_origin, out_size, in_origin, in_size, pad, bn_scale=None, bn_shift=None,
      bn_mean=None, out_ncdhw=False, in_c4=False, absmax=None, y_bound=None, per_lane=False, s2_lds=False):
    _eager_only("conv3d_region", y_bound=y_bound)
    if out_ncdhw:
        return x.new_empty((x.shape[0], weight.shape[1]) + tuple(out_size), dtype=_F32)
    return x.new_empty((x.shape[0],) + tuple(out_size) + (weight.shape[1],), dtype=_F32)


BOUND_WORDS = 2048   # MVS_BOUND_WORDS (64 slots, one per 128-byte line)


def bound_words(n, device):
    """n zeroed bound-word sets (int32 [n, MVS_BOUND_WORDS]) -- one memset for a forward's tensors."""
    return torch.zeros((n, BOUND_WORDS), device=device, dtype=torch.int32)


def _bound_ptr(t):
    if t is None:
        return None
    if t.dtype != torch.int32 or t.numel() != BOUND_WORDS or not t.is_contiguous():
        raise ValueError("bound words: a contiguous int32 tensor of %d words" % BOUND_WORDS)
    return _lib.ptr(t)


def region_split_fragments(weight, device):
    """(split-fp16 MFMA fragments on ``device``, exponent) of a region convolution's weight
    [27][c_out][c_in] (region_weight's layout), formed on the host by mvs_conv3d_region_split_weights."""
    lib = _lib.load()
    w = weight.detach().to(device="cpu", dtype=_F32).contiguous()
    _, cout, cin = w.shape
    kb = 14 if cin == 16 else 27 * (cin // 32)
    frag = torch.empty((kb * (cout // 16) * 2 * 64 * 8,), dtype=torch.int16)
    e = ctypes.c_int(0)
    st = lib.mvs_conv3d_region_split_weights(_lib.ptr(w), cin, cout, _lib.ptr(frag), ctypes.byref(e))
    _lib.check(st, "mvs_conv3d_region_split_weights")
    return frag.to(device), e.value


# (the bound words are raised in place; not declared as a mutation: torch's ADInplaceOrView wrapper
# indexes every declared mutable argument positionally, which fails for an omitted trailing default)
@torch.library.custom_op("mvs::conv3d_region_split", mutates_args=())
def conv3d_region_split(x: torch.Tensor, x2: Optional[torch.Tensor], weight: torch.Tensor, mode: int,
                        dims: list[int], out_origin: list[int], out_size: list[int], in_origin: Optional[list[int]],
                        in_size: Optional[list[int]], pad: Optional[list[int]], x_bound: Optional[torch.Tensor],
                        x2_bound: Optional[torch.Tensor], y_bound: Optional[torch.Tensor],
                        bn_scale: Optional[torch.Tensor] = None, bn_shift: Optional[torch.Tensor] = None,
                        bn_mean: Optional[torch.Tensor] = None, out_ncdhw: bool = False,
                        per_lane: bool = False, y_addend: Optional[torch.Tensor] = None,
                        store_origin: Optional[list[int]] = None, store_size: Optional[list[int]] = None,
                        stats: Optional[torch.Tensor] = None, in_bn: Optional[torch.Tensor] = None) -> torch.Tensor:
    """conv3d_region's CONV_S1 / CONV_T2 convolutions on the f16 matrix cores with split operands
    (mvs_conv3d_region_split_fwd, csrc/conv3d_region_split.hip): same geometry, layouts and epilogue;
    the input scaled by its bound words ``x_bound`` (+ ``x2_bound`` for the sum x + x2), ``y_bound``
    (zeroed words or None) raised to max|y|.  ``y_addend``: added to the output after BN + ReLU (same
    shape and layout as y).  CONV_S2: x is the split cost volume (int32 [B, 8, D, H, W,
    4], or a box of it with in_origin / in_size), x_bound its 8 bound words.  ``store_origin`` /
    ``store_size``: y holds only that box of the output region (the rest is computed, not stored);
    ``stats``: float64 [split_stats_slots, 2, c_out] receiving per-workgroup sums over the whole
    output region (conv3d_region_split_sums).  ``in_bn`` (CONV_T2, 64 -> 32 / 32 -> 16): fp32 [6, c_in]
    = (scale, shift, mean) of x then x2 -- the input is relu(BN(x)) [+ relu(BN(x2))], the bound words
    bound the raw tensors; also CONV_S1 16 -> 16 / 32 -> 32 (its LDS kernel), x only.  fp32-level error
    (DESIGN.md §3.8).  Inference only."""
    _require_gpu(x, "x")
    lib = _lib.load()
    flags = (_lib.MVS_CONV_OUT_NCDHW if out_ncdhw else 0) | (_lib.MVS_CONV_PER_LANE if per_lane else 0)
    if mode == CONV_S2:
        if x.dtype != torch.int32 or x.dim() != 6 or x_bound is None or x_bound.numel() != 8:
            raise ValueError("CONV_S2: the split cost volume [B, 8, D, H, W, 4] int32 and its 8 bound words")
        flags |= _lib.MVS_CONV_IN_C4 | _lib.MVS_CONV_IN_SPLIT
        x = x.contiguous()
    else:
        x = x.to(_F32).contiguous()
    if x2 is not None:
        x2 = x2.to(_F32).contiguous()
    dev = x.device
    frag, ew = derived("region_split", (weight,), lambda wt: region_split_fragments(wt, dev), dev)
    _, cout, cin = weight.shape
    b = x.shape[0]
    bn = [t if t is None else t.to(device=dev, dtype=_F32).contiguous() for t in (bn_scale, bn_shift, bn_mean)]
    if any(t is None for t in bn) and not all(t is None for t in bn):
        raise ValueError("bn_scale, bn_shift and bn_mean go together")
    ysz = tuple(out_size if store_size is None else store_size)
    shape = (b, cout) + ysz if out_ncdhw else (b,) + ysz + (cout,)
    y = torch.empty(shape, device=dev, dtype=_F32)
    xb = (_lib.ptr(x_bound.contiguous()) if mode == CONV_S2 else _bound_ptr(x_bound))
    if stats is not None:
        slots = split_stats_slots(mode, b, cin, cout, out_size, per_lane, x2 is not None, in_bn is not None)
        if stats.dtype != torch.float64 or stats.numel() != slots * 2 * cout or not stats.is_contiguous():
            raise ValueError("stats: a contiguous float64 tensor of %d x 2 x %d" % (slots, cout))
    ya = None
    if y_addend is not None:
        if tuple(y_addend.shape) != tuple(y.shape) or y_addend.dtype != _F32 or not y_addend.is_contiguous():
            raise ValueError("y_addend: a contiguous fp32 tensor of the output's shape")
        ya = _lib.ptr(y_addend)
    st = lib.mvs_conv3d_region_split_fwd(int(mode), flags, _lib.ptr(x),
                                         None if x2 is None else _lib.ptr(x2), _lib.ptr(frag), int(ew), _lib.ptr(y),
                                         b, cin, cout, _ints3(dims), _ints3(out_origin), _ints3(out_size),
                                         None if in_origin is None else _ints3(in_origin),
                                         None if in_size is None else _ints3(in_size),
                                         None if pad is None else _ints3(pad),
                                         *[None if t is None else _lib.ptr(t) for t in bn], xb,
                                         _bound_ptr(x2_bound), _bound_ptr(y_bound), ya,
                                         None if store_origin is None else _ints3(store_origin),
                                         None if store_size is None else _ints3(store_size),
                                         None if stats is None else _lib.ptr(stats), None, None,
                                         None if in_bn is None else _lib.ptr(in_bn.contiguous()),
                                         _lib.stream_handle(dev))
    _lib.check(st, "mvs_conv3d_region_split_fwd")
    return y


def conv_s2_split_multi_sums(cv, weights, dims, out_origin, out_size, pad, bound, y_bound=None):
    """Train mode's conv_1_0, conv_2_0 and conv_3_0 (16 / 32 / 64 channels, model.py:78-80) over ONE
    region of the split cost volume in one launch (mvs_conv3d_region_split_fwd, c_out = 112: the
    volume's A fragments are loaded once for all three), without BN, with the per-channel float64 batch
    sums formed in the epilogue: returns [(y, s1, s2)] per conv, y channels-last on the region.
    ``weights``: the three region weights [27, c_k, 32] (region_weight); ``y_bound``: None or zeroed
    bound words raised to the max |y| over the three outputs."""
    _require_gpu(cv, "cv")
    lib = _lib.load()
    if cv.dtype != torch.int32 or cv.dim() != 6 or bound is None or bound.numel() != 8:
        raise ValueError("the split cost volume [B, 8, D, H, W, 4] int32 and its 8 bound words")
    if [w.shape[1] for w in weights] != [16, 32, 64] or any(w.shape[2] != 32 for w in weights):
        raise ValueError("weights: region weights of c_out 16, 32, 64 over 32 input channels")
    cv = cv.contiguous()
    dev = cv.device
    frag, ew = derived("region_split_multi", tuple(weights),
                       lambda *ws: region_split_fragments(torch.cat([w.detach() for w in ws], 1), dev), dev)
    b = cv.shape[0]
    ys = [torch.empty((b,) + tuple(out_size) + (c,), device=dev, dtype=_F32) for c in (16, 32, 64)]
    slots = split_stats_slots(CONV_S2, b, 32, 112, out_size)
    st = torch.empty((slots, 2, 112), device=dev, dtype=torch.float64)
    flags = _lib.MVS_CONV_IN_C4 | _lib.MVS_CONV_IN_SPLIT
    rc = lib.mvs_conv3d_region_split_fwd(CONV_S2, flags, _lib.ptr(cv), None, _lib.ptr(frag), int(ew), _lib.ptr(ys[0]),
                                         b, 32, 112, _ints3(dims), _ints3(out_origin), _ints3(out_size), None, None,
                                         _ints3(pad), None, None, None, _lib.ptr(bound.contiguous()), None,
                                         _bound_ptr(y_bound), None, None, None, _lib.ptr(st), _lib.ptr(ys[1]),
                                         _lib.ptr(ys[2]), None,
                                         _lib.stream_handle(dev))
    _lib.check(rc, "mvs_conv3d_region_split_fwd")
    s = st.sum(0)
    return [(ys[k], s[0, lo:hi], s[1, lo:hi]) for k, (lo, hi) in enumerate(((0, 16), (16, 48), (48, 112)))]


def split_stats_slots(mode, batch, c_in, c_out, out_size, per_lane=False, two_inputs=False, in_bn=False):
    """Sum slots (workgroups) of a conv3d_region_split launch (mvs_conv3d_region_split_stats_slots)."""
    flags = ((_lib.MVS_CONV_PER_LANE if per_lane else 0) | (_lib.MVS_CONV_SUM_INPUT if two_inputs else 0)
             | (_lib.MVS_CONV_IN_BN if in_bn else 0))
    n = _lib.load().mvs_conv3d_region_split_stats_slots(int(mode), flags, int(batch), int(c_in), int(c_out),
                                                       _ints3(out_size))
    if n <= 0:
        raise ValueError("mvs_conv3d_region_split_stats_slots: %d" % n)
    return int(n)


def conv3d_region_split_sums(x, x2, weight, mode, dims, out_origin, out_size, in_origin, in_size, pad, x_bound,
                             x2_bound=None, y_bound=None, out_ncdhw=False, store_origin=None, store_size=None,
                             x_bn=None, x2_bn=None):
    """conv3d_region_split without the BN epilogue (train mode's raw output), with the per-channel
    float64 (sum, sum of squares) over the whole output region formed in the kernel's epilogue:
    returns (y, s1, s2), y holding the store box (default: the output region).  Replaces
    channel_stats(y) on the output: no second pass over it, and y may hold only the part the next layer
    reads.  ``x_bn`` / ``x2_bn``: (scale, shift, mean) -- the input is relu(BN(x)) [+
    relu(BN(x2))] (CONV_T2's LDS kernel: the BN + ReLU passes folded into its staging)."""
    b, cout, cin = x.shape[0], weight.shape[1], weight.shape[2]
    in_bn = None
    if x2 is not None and (x_bn is None) != (x2_bn is None):
        raise ValueError("x_bn and x2_bn go together when x2 is given")
    if x_bn is not None:
        ones, zeros = torch.ones(cin, device=x.device), torch.zeros(cin, device=x.device)
        rows = list(x_bn) + (list(x2_bn) if x2_bn is not None else [ones, zeros, zeros])
        in_bn = torch.stack([t.detach().to(device=x.device, dtype=_F32).reshape(cin) for t in rows])
    slots = split_stats_slots(mode, b, cin, cout, out_size, False, x2 is not None, in_bn is not None)
    st = torch.empty((slots, 2, cout), device=x.device, dtype=torch.float64)
    y = conv3d_region_split(x, x2, weight, mode, dims, out_origin, out_size, in_origin, in_size, pad, x_bound,
                            x2_bound, y_bound, out_ncdhw=out_ncdhw, store_origin=store_origin,
                            store_size=store_size, stats=st, in_bn=in_bn)
    s = st.sum(0)
    return y, s[0], s[1]


@conv3d_region_split.register_fake
def _(x, x2, weight, mode, dims, out_origin, out_size, in_origin, in_size, pad, x_bound, x2_bound, y_bound,
      bn_scale=None, bn_shift=None, bn_mean=None, out_ncdhw=False, per_lane=False, y_addend=None,
      store_origin=None, store_size=None, stats=None, in_bn=None):
    _eager_only("conv3d_region_split", y_bound=y_bound, stats=stats)
    size = tuple(out_size if store_size is None else store_size)
    if out_ncdhw:
        return x.new_empty((x.shape[0], weight.shape[1]) + size, dtype=_F32)
    return x.new_empty((x.shape[0],) + size + (weight.shape[1],), dtype=_F32)


# ----------------------------------------------------------------------------------------------
# train-mode BatchNorm pieces of the regulariser (csrc/channel_ops.hip; forward_live_train)
# ----------------------------------------------------------------------------------------------
def channel_stats(x: torch.Tensor, channels_last: bool):
    """Per-channel (sum, sum of squares) of x in float64 [C] each: channels on the last dim
    (channels_last) or on dim 1 (NCDHW).  Slot-owned partial sums (no atomics) added in a fixed
    order: bit-identical run to run.  Inference only."""
    _require_gpu(x, "x")
    lib = _lib.load()
    x = x.to(_F32).contiguous()
    c = x.shape[-1] if channels_last else x.shape[1]
    vox = x.numel() // (x.shape[0] * c)
    layout = _lib.MVS_LAYOUT_CHANNELS_LAST if channels_last else 0
    slots = lib.mvs_channel_stats_slots(layout, x.shape[0], c, vox)
    st = torch.empty((max(slots, 1), 2, c), device=x.device, dtype=torch.float64)
    rc = lib.mvs_channel_stats(_lib.ptr(x), layout, x.shape[0], c, vox, _lib.ptr(st), _lib.stream_handle(x.device))
    _lib.check(rc, "mvs_channel_stats")
    s = st.sum(0)
    return s[0], s[1]


def bn_train_params(bn, s1, s2, count, border=None):
    """Train-mode BatchNorm parameters [3, C] = (scale, shift, mean) from the float64 batch sums s1, s2
    over ``count`` elements, updating bn's running statistics and num_batches_tracked (mvs_bn_train_params,
    csrc/channel_ops.hip: one launch for what model._bn_train does in ~12 device ops).  ``border``: None
    or (U [C, C_prev, K] float64, counts [K] float64, prev [3, C_prev]) -- conv_k_1's border-class term
    (model._border_class_sums) with the previous BN's constant relu(BN(0)) formed from its parameters
    ``prev``.  bn.momentum must be set (None: the cumulative average, model._bn_train)."""
    lib = _lib.load()
    if bn.momentum is None:
        raise ValueError("bn_train_params: momentum=None (cumulative average) is model._bn_train's")
    c = s1.numel()
    if (s1.dim() == 1 and s2.dim() == 1 and s1.is_contiguous() and s2.is_contiguous()
            and s1.dtype == torch.float64 and s2.dtype == torch.float64
            and s1.untyped_storage().data_ptr() == s2.untyped_storage().data_ptr()
            and s2.data_ptr() == s1.data_ptr() + 8 * c):
        sums = torch.as_strided(s1, (2, c), (c, 1))   # the rows of one [2, C] sum tensor
    else:
        sums = torch.stack((s1.double(), s2.double()))
    dev = sums.device
    f = lambda t: t.detach().to(device=dev, dtype=_F32).contiguous()
    wt, bias = f(bn.weight), f(bn.bias)
    params = torch.empty((3, c), device=dev, dtype=_F32)
    track = bn.running_mean is not None
    if track and not (bn.running_mean.is_contiguous() and bn.running_mean.dtype == _F32
                      and bn.running_var.is_contiguous() and bn.running_var.dtype == _F32):
        raise ValueError("bn_train_params: contiguous fp32 running statistics expected")
    bu = bc = prev = None
    cp = ncls = 0
    if border is not None:
        bu, bc, prev = border
        cp, ncls = bu.shape[1], bu.shape[2]
        if bu.shape[0] != c or bc.numel() != ncls or tuple(prev.shape) != (3, cp):
            raise ValueError("border: U [C, C_prev, K], counts [K], prev [3, C_prev]")
        prev = prev.contiguous()
    nbt = bn.num_batches_tracked if track and bn.num_batches_tracked is not None else None
    pt = lambda t: None if t is None else _lib.ptr(t)
    st = lib.mvs_bn_train_params(_lib.ptr(sums.contiguous()), c, float(count), pt(bu), pt(bc), cp, ncls, pt(prev),
                                 _lib.ptr(wt), _lib.ptr(bias), pt(bn.running_mean if track else None),
                                 pt(bn.running_var if track else None), pt(nbt), float(bn.momentum), float(bn.eps),
                                 _lib.ptr(params), _lib.stream_handle(dev))
    _lib.check(st, "mvs_bn_train_params")
    return params


def bn_relu_(x: torch.Tensor, channels_last: bool, scale, shift, mean, r=None, r_bn=None, y_bound=None) -> torch.Tensor:
    """In place: x = relu((x - mean) * scale + shift) [+ relu(BN_r(r))], channels on the last dim
    (channels_last) or dim 1; r_bn = (scale, shift, mean) of r.  x must be contiguous fp32.
    ``y_bound``: zeroed bound words raised to max of the result."""
    _require_gpu(x, "x")
    lib = _lib.load()
    if not x.is_contiguous() or x.dtype != _F32:
        raise ValueError("bn_relu_ works in place on a contiguous fp32 tensor")
    c = x.shape[-1] if channels_last else x.shape[1]
    vox = x.numel() // (x.shape[0] * c)
    f = lambda t: t.to(device=x.device, dtype=_F32).contiguous()
    sc, sh, mu = f(scale), f(shift), f(mean)
    rr = rs = None
    if r is not None:
        rr = f(r)
        if rr.shape != x.shape:
            raise ValueError("r must have x's shape")
        rs = [f(t) for t in r_bn]
    pt = lambda t: None if t is None else _lib.ptr(t)
    rc = lib.mvs_bn_relu(_lib.ptr(x), _lib.MVS_LAYOUT_CHANNELS_LAST if channels_last else 0, x.shape[0], c, vox,
                         pt(sc), pt(sh), pt(mu), pt(rr), *(pt(t) for t in (rs or (None, None, None))), _lib.ptr(x),
                         _bound_ptr(y_bound), _lib.stream_handle(x.device))
    _lib.check(rc, "mvs_bn_relu")
    return x


def softmax_depth(x: torch.Tensor) -> torch.Tensor:
    """nn.Softmax(2) of the regulariser's [B, 1, D, h, w] output (model.py:97) on the HIP kernel.
    Inference only."""
    _require_gpu(x, "x")
    lib = _lib.load()
    if x.dim() != 5 or x.shape[1] != 1:
        raise ValueError("softmax_depth expects [B, 1, D, h, w], got %s" % (tuple(x.shape),))
    x = x.to(_F32).contiguous()
    y = torch.empty_like(x)
    b, _, d, h, w = x.shape
    rc = lib.mvs_softmax_depth_fwd(_lib.ptr(x), b, d, h, w, _lib.ptr(y), _lib.stream_handle(x.device))
    _lib.check(rc, "mvs_softmax_depth_fwd")
    return y


def _per_sample(t, batch, device):
    """d_min / d_int as a contiguous fp32 [batch] device tensor (one value per sample, or one for all)."""
    t = t.to(device=device, dtype=_F32).reshape(-1)
    if t.numel() == 1:
        t = t.expand(batch)
    if t.numel() != batch:
        raise ValueError("d_min / d_int: one value per sample (%d) or one in all, got %d" % (batch, t.numel()))
    return t.contiguous()


def refine_input(initial_depth: torch.Tensor, d_min: torch.Tensor, d_int: torch.Tensor, d_num: int,
                 d_scale: float, ref_img: torch.Tensor) -> torch.Tensor:
    """torch.cat(((initial_depth - d_min) / ((d_int * d_num) * d_scale), ref_img), 1) (model.py:195-199)
    in one HIP launch (mvs_refine_input_fwd), bit-equal to the torch sequence.  Inference only."""
    _require_gpu(initial_depth, "initial_depth")
    lib = _lib.load()
    b, c, h, w = initial_depth.shape
    if c != 1 or tuple(ref_img.shape) != (b, 3, h, w):
        raise ValueError("initial_depth [B, 1, h, w] and ref_img [B, 3, h, w] expected, got %s, %s"
                         % (tuple(initial_depth.shape), tuple(ref_img.shape)))
    dev = initial_depth.device
    ini = initial_depth.to(_F32).contiguous()
    img = ref_img.to(device=dev, dtype=_F32).contiguous()
    dm, di = _per_sample(d_min, b, dev), _per_sample(d_int, b, dev)
    out = torch.empty((b, 4, h, w), device=dev, dtype=_F32)
    rc = lib.mvs_refine_input_fwd(_lib.ptr(ini), _lib.ptr(dm), _lib.ptr(di), b, h, w, int(d_num), float(d_scale),
                                  _lib.ptr(img), _lib.ptr(out), _lib.stream_handle(dev))
    _lib.check(rc, "mvs_refine_input_fwd")
    return out


def refine_output(conv: torch.Tensor, refine_in: torch.Tensor, d_min: torch.Tensor, d_int: torch.Tensor,
                  d_num: int, d_scale: float) -> torch.Tensor:
    """((conv + refine_in[:, 0]) * ((d_int * d_num) * d_scale)) + d_min -- the refinement's residual
    add and the rescale (model.py:150, 204-205) in one HIP launch (mvs_refine_output_fwd), bit-equal to
    the torch sequence.  Inference only."""
    _require_gpu(conv, "conv")
    lib = _lib.load()
    b, c, h, w = conv.shape
    if c != 1 or tuple(refine_in.shape) != (b, 4, h, w):
        raise ValueError("conv [B, 1, h, w] and refine_in [B, 4, h, w] expected, got %s, %s"
                         % (tuple(conv.shape), tuple(refine_in.shape)))
    dev = conv.device
    cv = conv.to(_F32).contiguous()
    ri = refine_in.to(_F32).contiguous()
    dm, di = _per_sample(d_min, b, dev), _per_sample(d_int, b, dev)
    out = torch.empty((b, 1, h, w), device=dev, dtype=_F32)
    rc = lib.mvs_refine_output_fwd(_lib.ptr(cv), _lib.ptr(ri), _lib.ptr(dm), _lib.ptr(di), b, h, w, int(d_num),
                                   float(d_scale), _lib.ptr(out), _lib.stream_handle(dev))
    _lib.check(rc, "mvs_refine_output_fwd")
    return out


def depth_hypotheses(d_min: torch.Tensor, d_int: torch.Tensor, d_num: int, d_scale: float) -> torch.Tensor:
    """homography.py:24-26 d_batch_0 [B, d_num, 1, 1] = d_min + d_scale * d_int * k in one HIP launch
    (mvs_depth_hypotheses_fwd), bit-equal to the torch expression.  d_min, d_int [B, 1, 1, 1] (or one
    value for all samples) on the device; inference only."""
    _require_gpu(d_min, "d_min")
    lib = _lib.load()
    b = d_min.shape[0] if d_min.numel() > 1 else d_int.reshape(-1).shape[0]
    dev = d_min.device
    dm, di = _per_sample(d_min, b, dev), _per_sample(d_int, b, dev)
    out = torch.empty((b, int(d_num), 1, 1), device=dev, dtype=_F32)
    rc = lib.mvs_depth_hypotheses_fwd(_lib.ptr(dm), _lib.ptr(di), b, int(d_num), float(d_scale), _lib.ptr(out),
                                      _lib.stream_handle(dev))
    _lib.check(rc, "mvs_depth_hypotheses_fwd")
    return out
