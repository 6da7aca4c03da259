"""CPU: the C-ABI library exists, loads, and exports every entry point include/*.h declares.

No kernel is launched here (no GPU); only host-side functions that touch no device are called.
"""
import glob
import os
import re

import pytest

from conftest import REPO


def _declared():
    names = []
    for h in glob.glob(os.path.join(REPO, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names += re.findall(r"^\s*(?:const\s+)?[\w\*\s]+?\b(mvs_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_abi():
    names = _declared()
    assert "mvs_cost_volume_fwd" in names and "mvs_cost_volume_bwd" in names
    assert len(names) == 45, names


def test_library_exports_every_declared_symbol():
    from mvs_amd import _lib
    lib = _lib.load()
    for name in _declared():
        assert hasattr(lib, name), name
    assert set(_declared()) == set(_lib.SIGNATURES), "ctypes bindings out of sync with the header"


def test_host_only_entry_points():
    from mvs_amd import _lib
    lib = _lib.load()
    assert lib.mvs_abi_version() == _lib.ABI_VERSION == 24
    assert lib.mvs_status_string(0) == b"ok"
    assert lib.mvs_status_string(-2).startswith(b"n_views")
    assert lib.mvs_sampling_workspace_bytes(12, 192) == 12 * 192 * 9 * 4
    assert lib.mvs_sampling_workspace_bytes(0, 192) == 0


def test_invalid_arguments_rejected_before_any_launch():
    """Argument validation returns an error code without touching the device."""
    import ctypes
    from mvs_amd import _lib
    lib = _lib.load()
    null = ctypes.c_void_p(0)
    fake = ctypes.c_void_p(0x1000)
    # null pointers
    assert lib.mvs_cost_volume_fwd(null, fake, fake, fake, fake, fake, 1, 3, 32, 128, 160, 0, 48,
                                   25.0, fake, fake, null) == -1
    # unsupported view count
    assert lib.mvs_cost_volume_fwd(fake, fake, fake, fake, fake, fake, 1, 17, 32, 128, 160, 0, 48,
                                   25.0, fake, fake, null) == -2
    # degenerate image (kornia's (w-1) normalisation needs w, h >= 2)
    assert lib.mvs_cost_volume_fwd(fake, fake, fake, fake, fake, fake, 1, 3, 32, 1, 160, 0, 48,
                                   25.0, fake, fake, null) == -1
    # per-image index space
    assert lib.mvs_cost_volume_fwd(fake, fake, fake, fake, fake, fake, 1, 3, 70000, 128, 256, 0, 4,
                                   25.0, fake, fake, null) == -3
    # 32-bit buffer descriptors of the packed kernels: C=4 with hw = 2^28 passes the per-image
    # element bound (C*hw < 2^31) but not the descriptor byte counts
    assert lib.mvs_cost_volume_fwd(fake, fake, fake, fake, fake, fake, 1, 3, 4, 16384, 16384, 0, 4,
                                   25.0, fake, fake, null) == -3
    # 8 views of 32 channels at 2048x2048 features: 8 * 8 * 2050 * 2050 * 16 B > 2^31
    assert lib.mvs_cost_volume_fwd(fake, fake, fake, fake, fake, fake, 1, 8, 32, 2048, 2048, 0, 4,
                                   25.0, fake, fake, null) == -3
    assert lib.mvs_extract_depth_map_fwd(fake, fake, 1, 48, 8, 8, 0, fake, null) == -1
    # backward: missing backward workspace (needed for n_views > 1), bad geometry
    assert lib.mvs_cost_volume_bwd(fake, fake, fake, 1, 3, 32, 128, 160, 48, 0, null, fake, null) == -1
    assert lib.mvs_cost_volume_bwd(fake, fake, fake, 1, 17, 32, 128, 160, 48, 0, fake, fake, null) == -2
    assert lib.mvs_cost_volume_bwd(fake, fake, fake, 1, 3, 32, 128, 160, 48, 2, fake, fake, null) == -1
    assert lib.mvs_cost_volume_bwd_workspace_bytes(1, 3, 32, 128, 160, 0, 0) == 0
    assert lib.mvs_cost_volume_bwd_workspace_bytes(1, 3, 32, 128, 160, 48, 2) == 0      # unknown flag
    # deterministic mode: 64-bit accumulators for every feature element + reference-view partials +
    # scalars; the default mode needs no accumulators
    det = lib.mvs_cost_volume_bwd_workspace_bytes(4, 3, 32, 128, 160, 192, 1)
    dflt = lib.mvs_cost_volume_bwd_workspace_bytes(4, 3, 32, 128, 160, 192, 0)
    assert det - dflt >= 12 * 32 * 128 * 160 * 8
    # the channel-quad store (16 B per voxel quad, up to 8 planes per descriptor) wraps 32-bit offsets
    # at hw >= 2^25: C=4, V=2, 6000x6000 passes every other bound but must be refused, not dropped
    c4_out = ctypes.c_void_p(1 << 20)
    assert lib.mvs_cost_volume_fwd_c4(fake, fake, fake, fake, fake, fake, 1, 2, 4, 6000, 6000, 0, 4, 25.0,
                                      fake, c4_out, null, None, None) == -3
    # deterministic partial-sum slots of the BN statistics (every slot written, none zeroed)
    assert lib.mvs_channel_stats_slots(0, 2, 8, 1000) >= 2
    assert lib.mvs_channel_stats_slots(1, 2, 16, 1000) >= 1
    assert lib.mvs_channel_stats_slots(2, 2, 16, 1000) == 0 and lib.mvs_channel_stats_slots(0, 0, 8, 10) == 0
    # train-mode BN pieces: channels-last needs 4 | C with C / 4 a power of two, and 16-B alignment
    assert lib.mvs_channel_stats(fake, 1, 2, 24, 100, fake, null) == -1
    assert lib.mvs_channel_stats(ctypes.c_void_p(20), 1, 2, 16, 100, fake, null) == -1
    assert lib.mvs_channel_stats(fake, 2, 2, 16, 100, fake, null) == -1
    assert lib.mvs_channel_stats(fake, 0, 2, 16, 0, fake, null) == -1
    assert lib.mvs_bn_relu(fake, 0, 2, 16, 100, fake, fake, None, None, None, None, None, fake, None, null) == -1
    assert lib.mvs_bn_relu(fake, 0, 2, 16, 100, fake, fake, fake, fake, None, fake, fake, fake, None, null) == -1
    # the split region convs' sum slots: host-only arithmetic over the launch geometry
    size = (ctypes.c_int * 3)(26, 18, 22)
    s1 = lib.mvs_conv3d_region_split_stats_slots(0, 0, 2, 16, 16, size)                    # LDS kernel tiles
    assert s1 == 2 * 2 * 5 * 4   # ceil(22 / 16) x ceil(18 / 4) x ceil(26 / 8) tiles x batch 2
    t2 = lib.mvs_conv3d_region_split_stats_slots(2, 0, 2, 64, 32, size)
    assert t2 > 0 and t2 % (8 * 2 * 8) == 0   # (row chunks rounded to 8 XCDs) x 8 classes x batch
    assert lib.mvs_conv3d_region_split_stats_slots(0, _lib.MVS_CONV_PER_LANE, 2, 16, 16, size) != s1
    assert lib.mvs_conv3d_region_split_stats_slots(3, 0, 2, 16, 16, size) == -1
    assert lib.mvs_conv3d_region_split_stats_slots(0, 0, 0, 16, 16, size) == -1


def test_build_is_gfx950_in_tree():
    from mvs_amd import _build
    assert _build.ARCH == "gfx950" or os.environ.get("MVS_OFFLOAD_ARCH")
    assert os.path.dirname(_build.OUTPUT).startswith(REPO)
    data = open(_build.OUTPUT, "rb").read()
    assert b"gfx950" in data
