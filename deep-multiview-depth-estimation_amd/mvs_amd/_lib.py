"""ctypes binding of the C ABI in ``include/mvs_cost_volume.h`` (libmvs_cost_volume.so).

The library is built in-tree by ``mvs_amd._build.build_library()`` (called from
``__graft_entry__.build()``) and travels to the GPU box as a file next to this module.  There is
no fallback: if the library is missing or was built for another ABI, every op raises
``MVSLibraryError`` -- the product path never drops to a CPU or eager-PyTorch implementation.

``torch`` is imported before the library is loaded on purpose: torch ships its own
``libamdhip64.so.7`` and the dynamic loader then resolves the library's HIP dependency to that
same runtime (one HIP runtime per process, so torch's streams are valid here).
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libmvs_cost_volume.so"
# MVS_LIB_PATH: load another build of the same ABI (A/B kernel experiments, tools/gpu_*_ab.sh)
LIB_PATH = os.environ.get("MVS_LIB_PATH") or os.path.join(_HERE, LIB_NAME)
ABI_VERSION = 24

MVS_OK = 0
MVS_BWD_DETERMINISTIC = 1
MVS_LAYOUT_CHANNELS_LAST = 1
MVS_CONV_S1, MVS_CONV_S2, MVS_CONV_T2 = 0, 1, 2
MVS_CONV_OUT_NCDHW = 1
MVS_CONV_PER_LANE = 32
MVS_CONV_S2_LDS = 256
MVS_CONV_SUM_INPUT = 64
MVS_CONV_IN_BN = 128
MVS_CONV_IN_C4 = 2
MVS_CONV_WINO_Z = 4
MVS_CONV_IN_BF16 = 8
MVS_CONV_IN_SPLIT = 16
MVS_DECONV_WEIGHT_TAPS = 2
STATUS = {0: "ok", -1: "invalid argument", -2: "unsupported n_views", -3: "too large",
          -4: "HIP runtime error"}

_c_int, _c_float, _p = ctypes.c_int, ctypes.c_float, ctypes.c_void_p

# name -> (restype, argtypes); mirrors include/mvs_cost_volume.h
SIGNATURES = {
    "mvs_abi_version": (_c_int, []),
    "mvs_status_string": (ctypes.c_char_p, [_c_int]),
    "mvs_sampling_workspace_bytes": (ctypes.c_size_t, [_c_int, _c_int]),
    "mvs_cost_volume_workspace_bytes": (ctypes.c_size_t, [_c_int, _c_int, _c_int, _c_int, _c_int,
                                                           _c_int]),
    "mvs_plane_sampling": (_c_int, [_p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int, _c_int,
                                    _c_int, _c_float, _p, _p]),
    "mvs_cost_volume_fwd": (_c_int, [_p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int,
                                     _c_int, _c_int, _c_int, _c_float, _p, _p, _p]),
    "mvs_cost_volume_fwd_timed": (_c_int, [_p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int,
                                           _c_int, _c_int, _c_int, _c_float, _p, _p, _p, _p, _p]),
    "mvs_cost_volume_fwd_c4": (_c_int, [_p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int,
                                        _c_int, _c_int, _c_int, _c_float, _p, _p, _p, _p, _p]),
    "mvs_cost_volume_fwd_c4_absmax": (_c_int, [_p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int,
                                               _c_int, _c_int, _c_int, _c_float, _p, _p, _p, _p, _p, _p]),
    "mvs_conv3d_k3_split_fwd": (_c_int, [_p, _c_int, _p, _c_int, _p, _p] + [_c_int] * 4 + [_p] * 4),
    "mvs_cost_volume_fwd_c4_split": (_c_int, [_p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int,
                                              _c_int, _c_int, _c_int, _c_float, _p, _p, _p, _p, _p, _p]),
    "mvs_conv3d_split_weights": (_c_int, [_p, _p, _p]),
    "mvs_conv3d_s2_split_fwd": (_c_int, [_p, _c_int, _p, _c_int, _p, _p, _c_int] + [_p] * 8),
    "mvs_conv3d_s2_split_weights": (_c_int, [_p, _p, _p]),
    "mvs_split_head_fwd": (_c_int, [_p, _p, _c_int, _c_int, _c_int, _c_int, _p, _c_int, _p, _p, _p,
                                    _p, _c_int, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "mvs_cost_volume_head_fwd": (_c_int, [_p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int, _c_int,
                                          _c_int, _c_int, _c_float,
                                          _p, _c_int, _p, _p, _p, _p, _c_int, _p, _p, _p,
                                          _p, _p, _p, _p, _p,
                                          _p, _p, _p, _p, _p, _p, _p, _p]),
    "mvs_cost_volume_fwd_c4_bf16": (_c_int, [_p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int,
                                             _c_int, _c_int, _c_int, _c_float, _p, _p, _p, _p, _p]),
    "mvs_cost_volume_fwd_bf16": (_c_int, [_p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int,
                                          _c_int, _c_int, _c_int, _c_float, _p, _p, _p]),
    "mvs_homography_warp_fwd": (_c_int, [_p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int,
                                         _c_int, _c_int, _c_int, _c_float, _p, _p, _p]),
    "mvs_assemble_cost_volume_fwd": (_c_int, [_p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                                              _p, _p]),
    "mvs_cost_volume_bwd_workspace_bytes": (ctypes.c_size_t, [_c_int, _c_int, _c_int, _c_int,
                                                              _c_int, _c_int, _c_int]),
    "mvs_cost_volume_bwd": (_c_int, [_p, _p, _p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                                     _c_int, _p, _p, _p]),
    "mvs_extract_depth_map_fwd": (_c_int, [_p, _p, _c_int, _c_int, _c_int, _c_int, _c_int, _p,
                                           _p]),
    "mvs_normalize_images": (_c_int, [_p, _c_int, _c_int, _c_int, _p, _p, _p, _p]),
    "mvs_depth_threshold": (_c_int, [_p, ctypes.c_size_t, _c_float, _c_float, _p, _p]),
    "mvs_conv3d_k3_fwd": (_c_int, [_p, _c_int, _p, _p] + [_c_int] * 6 + [_p] * 6),
    "mvs_conv_head_fp32_fwd": (_c_int, [_p] + [_c_int] * 4 + [_p] * 17),
    "mvs_conv3d_k3_wgrad_workspace_bytes": (ctypes.c_size_t, [_c_int] * 5),
    "mvs_conv3d_k3_wgrad": (_c_int, [_p, _p] + [_c_int] * 6 + [_p, _p, _p]),
    "mvs_conv2d_fwd": (_c_int, [_p, _p, _p] + [_c_int] * 7 + [_p] * 5),
    "mvs_conv2d_split_weights": (_c_int, [_p, _c_int, _c_int, _c_int, _p, _p]),
    "mvs_conv2d_split_fwd": (_c_int, [_p, _p, _c_int, _p] + [_c_int] * 7 + [_p] * 6),
    "mvs_deconv3d_k3s2_fwd": (_c_int, [_p, _p] + [_c_int] * 10 + [_p] + [_c_int] * 6 + [_p] * 6),
    "mvs_conv3d_region_fwd": (_c_int, [_c_int, _c_int, _p, _p, _p, _p, _c_int, _c_int, _c_int] + [_p] * 12),
    "mvs_conv3d_region_split_weights": (_c_int, [_p, _c_int, _c_int, _p, _p]),
    "mvs_conv3d_region_split_fwd": (_c_int, [_c_int, _c_int, _p, _p, _p, _c_int, _p, _c_int, _c_int, _c_int]
                                    + [_p] * 20),
    "mvs_conv3d_region_split_stats_slots": (ctypes.c_longlong, [_c_int] * 5 + [_p]),
    "mvs_softmax_depth_fwd": (_c_int, [_p, _c_int, _c_int, _c_int, _c_int, _p, _p]),
    "mvs_depth_hypotheses_fwd": (_c_int, [_p, _p, _c_int, _c_int, _c_float, _p, _p]),
    "mvs_refine_input_fwd": (_c_int, [_p, _p, _p] + [_c_int] * 4 + [_c_float, _p, _p, _p]),
    "mvs_refine_output_fwd": (_c_int, [_p, _p, _p, _p] + [_c_int] * 4 + [_c_float, _p, _p]),
    "mvs_channel_stats_slots": (ctypes.c_size_t, [_c_int, _c_int, _c_int, ctypes.c_longlong]),
    "mvs_channel_stats": (_c_int, [_p, _c_int, _c_int, _c_int, ctypes.c_longlong, _p, _p]),
    "mvs_bn_relu": (_c_int, [_p, _c_int, _c_int, _c_int, ctypes.c_longlong] + [_p] * 10),
    "mvs_bn_train_params": (_c_int, [_p, _c_int, ctypes.c_double, _p, _p, _c_int, _c_int] + [_p] * 6
                            + [ctypes.c_double, ctypes.c_double, _p, _p]),
}


class MVSLibraryError(RuntimeError):
    """The HIP library is missing, stale, or a kernel call failed."""


_lib = None


def load():
    """Load (once) and return the ctypes handle; raises MVSLibraryError if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MVSLibraryError(
            "%s not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.mvs_abi_version() != ABI_VERSION:
        raise MVSLibraryError("ABI mismatch: library %d, bindings %d"
                              % (lib.mvs_abi_version(), ABI_VERSION))
    _lib = lib
    return lib


def check(status, what):
    if status != MVS_OK:
        raise MVSLibraryError("%s failed: %s (%d)" % (what, STATUS.get(status, "?"), status))


def ptr(t):
    """Device pointer of a tensor as a ctypes void*."""
    return ctypes.c_void_p(t.data_ptr())


def stream_handle(device):
    """The current torch (HIP) stream on ``device`` as a ctypes void*."""
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
