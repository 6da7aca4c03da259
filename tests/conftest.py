"""Shared pytest setup: import paths and the ``gpu`` marker.

``-m "not gpu"`` runs here (no GPU): oracle vs golden vectors, host logic, library load/exports,
gloo world_size-2 distributed logic.  ``-m gpu`` runs on an MI355X: parity of the HIP path
(through the C ABI) against the oracle and the golden vectors.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("deep-multiview-depth-estimation_amd", "oracle", os.path.join("tests", "golden")):
    p = os.path.join(REPO, sub)
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")
# MIOpen's find results for the regulariser's convolutions ship with the repo (tools/miopen_db,
# as bench.py uses them): without them the first full-volume cfg-2 convolutions search for minutes
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(REPO, "tools", "miopen_db"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) -- parity of the HIP path")


_CURRENT = ["-"]


@pytest.fixture(autouse=True)
def _heartbeat(request):
    """A line on the real stderr every 60 s naming the running test: the long end-to-end GPU tests
    (CPU oracle forwards, float64 autograd) stay visibly alive.  pytest.ini selects
    --capture=tee-sys (sys-level capture only), so fd 2 -- sys.__stderr__ -- is never redirected
    into pytest's capture file, with or without -s."""
    import threading
    import time
    _CURRENT[0] = request.node.nodeid
    if not getattr(_heartbeat, "started", False):
        _heartbeat.started = True

        def beat():
            t0 = time.time()
            while True:
                time.sleep(60)
                print("[heartbeat %4.0f s] %s" % (time.time() - t0, _CURRENT[0]), file=sys.__stderr__, flush=True)
        threading.Thread(target=beat, daemon=True).start()
    yield


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def load_golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name))


def record_parity(name, **values):
    """Measured parity numbers of a test (mask-flip fraction, share of pixels within 1e-4 of the
    oracle, error norms): printed as one "PARITY" JSON line and, when MVS_PARITY_OUT names a
    directory, written there as <name>.json (profiles/parity_*.json are collected this way)."""
    import json
    rec = {"test": name}
    rec.update({k: (float(v) if hasattr(v, "item") or isinstance(v, float) else v) for k, v in values.items()})
    print("PARITY " + json.dumps(rec))
    out = os.environ.get("MVS_PARITY_OUT")
    if out:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, name + ".json"), "w") as f:
            json.dump(rec, f, indent=1)
    return rec
