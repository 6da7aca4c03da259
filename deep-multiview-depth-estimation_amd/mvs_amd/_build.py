"""Build libmvs_cost_volume.so in-tree with hipcc for gfx950 (no JIT cache, no pip install)."""
import os
import shutil
import subprocess
import tempfile

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
REPO_ROOT = os.path.dirname(PKG_ROOT)
CSRC = os.path.join(PKG_ROOT, "csrc")
# one translation unit per kernel family + the C ABI (capi.hip); launchers.h declares the seams
SOURCES = [os.path.join(CSRC, f) for f in ("capi.hip", "plane_sampling.hip", "cost_volume_fwd.hip",
                                           "cost_volume_bwd.hip", "warp_variance.hip",
                                           "soft_argmin.hip", "dtu_input.hip",
                                           "conv3d_narrow.hip", "deconv3d_region.hip",
                                           "conv3d_region.hip", "channel_ops.hip", "conv2d_narrow.hip",
                                           "conv3d_split.hip", "conv3d_s2_split.hip", "cv_head.hip",
                                           "conv3d_region_split.hip", "conv2d_split.hip",
                                           "conv3d_wgrad.hip", "conv3d_s2_lds.hip")]
HEADERS = [os.path.join(REPO_ROOT, "include", "mvs_cost_volume.h"),
           os.path.join(CSRC, "common.h"), os.path.join(CSRC, "launchers.h"),
           os.path.join(CSRC, "packed.h"), os.path.join(CSRC, "sampling_matrix.h"),
           os.path.join(CSRC, "split.h")]
# per-source device flags, compiled as a separate object: the fused head (cv_head.hip) without packed
# fp32 VALU instructions -- with v_pk_{fma,add,mul}_f32 in its gather / variance code, the .z / .w halves of
# a producer item's variance came out wrong in a schedule-dependent share of launches (0 to 100 % of
# them across builds that only reorder the producer's instructions); the same builds without packed fp32:
# 0.  Elementwise identical arithmetic (a packed FMA is two fmaf): the outputs keep
# their bits.
SOURCE_FLAGS = {"cv_head.hip": ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]}
OUTPUT = os.path.join(_HERE, "libmvs_cost_volume.so")
ARCH = os.environ.get("MVS_OFFLOAD_ARCH", "gfx950")


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def build_library(force=False, verbose=False, extra_flags=(), output=None):
    """Compile the HIP sources into OUTPUT unless it is newer than every source/header."""
    out = output or OUTPUT
    if not force and not extra_flags and os.path.exists(out):
        newest = max(os.path.getmtime(p) for p in SOURCES + HEADERS)
        if os.path.getmtime(out) >= newest:
            return out
    base = [hipcc(), "-O3", "-std=c++17", "-Wno-pass-failed", "--offload-arch=%s" % ARCH, "-fPIC"]
    objs, srcs = [], []
    with tempfile.TemporaryDirectory(prefix="mvs_build_") as tmp:
        for src in SOURCES:
            flags = SOURCE_FLAGS.get(os.path.basename(src))
            if flags is None:
                srcs.append(src)
                continue
            obj = os.path.join(tmp, os.path.basename(src) + ".o")
            cmd = base + ["-c", "-o", obj] + list(extra_flags) + flags + [src]
            if verbose:
                print(" ".join(cmd))
            subprocess.check_call(cmd)
            objs.append(obj)
        cmd = base + ["-shared", "-parallel-jobs=%d" % min(8, os.cpu_count() or 1), "-o", out + ".tmp"] + \
            list(extra_flags) + srcs + ["-Wl,%s" % o for o in objs]   # (a bare .o would be read as HIP source)
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out
