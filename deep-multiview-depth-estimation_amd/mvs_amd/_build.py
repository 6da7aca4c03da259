"""Build libmvs_cost_volume.so in-tree with hipcc for gfx950 (no JIT cache, no pip install)."""
import os
import shutil
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
REPO_ROOT = os.path.dirname(PKG_ROOT)
SOURCES = [os.path.join(PKG_ROOT, "csrc", "mvs_cost_volume.hip")]
HEADERS = [os.path.join(REPO_ROOT, "include", "mvs_cost_volume.h")]
OUTPUT = os.path.join(_HERE, "libmvs_cost_volume.so")
ARCH = os.environ.get("MVS_OFFLOAD_ARCH", "gfx950")


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def build_library(force=False, verbose=False):
    """Compile the HIP sources into OUTPUT unless it is newer than every source/header."""
    if not force and os.path.exists(OUTPUT):
        newest = max(os.path.getmtime(p) for p in SOURCES + HEADERS)
        if os.path.getmtime(OUTPUT) >= newest:
            return OUTPUT
    cmd = [hipcc(), "-O3", "-std=c++17", "--offload-arch=%s" % ARCH, "-fPIC", "-shared",
           "-o", OUTPUT + ".tmp"] + SOURCES
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(OUTPUT + ".tmp", OUTPUT)
    return OUTPUT
