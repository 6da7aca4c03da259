"""Real DTU scan-1 camera sets built from ``dtu_scan1_cameras.npz`` (see extract_dtu_cameras.py).

Used for the golden fixtures, the GPU parity tests and ``bench.py``'s synthetic inputs
(SURVEY.md §8 d: real DTU geometry, synthetic pixels).  Pure numpy/torch; no reference code.
"""
import os

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
_NPZ = os.path.join(_HERE, "dtu_scan1_cameras.npz")
FIX_H, FIX_W = 128, 160    # K in the fixture is already at feature resolution


def load_fixture():
    z = np.load(_NPZ)   # plain arrays only (allow_pickle stays False)
    return {k: z[k] for k in z.files}


def _all_views(fx):
    """Per DTU view id (1..49): (K, R, T) taken from the sample whose reference view it is."""
    views = {}
    for s in range(fx["K"].shape[0]):
        vid = int(fx["view_ids"][s, 0])
        views[vid] = (fx["K"][s, 0], fx["R"][s, 0], fx["T"][s, 0])
    return views


def camera_batch(batch_size, n_views, h=FIX_H, w=FIX_W, first_sample=0):
    """K, R, T as torch fp32 [B*V,3,3], [B*V,3,3], [B*V,3,1] for B samples of V views.

    V == 3 uses the dataset's own triples (ref + pairs[0..1], ``data.py:237-246``); any other V uses
    the sample's ref view plus its V-1 nearest camera centres.  K rows are rescaled from the
    fixture's 160x128 feature grid to (w, h)."""
    fx = load_fixture()
    views = _all_views(fx)
    ids = sorted(views)
    centres = {v: (-views[v][1].T @ views[v][2]).ravel() for v in ids}
    Ks, Rs, Ts = [], [], []
    n_samples = fx["K"].shape[0]
    for b in range(batch_size):
        s = (first_sample + b) % n_samples
        if n_views == 3:
            K, R, T = fx["K"][s], fx["R"][s], fx["T"][s]
        else:
            ref = int(fx["view_ids"][s, 0])
            others = sorted((v for v in ids if v != ref),
                            key=lambda v: float(np.linalg.norm(centres[v] - centres[ref])))
            chosen = [ref] + others[: n_views - 1]
            K = np.stack([views[v][0] for v in chosen])
            R = np.stack([views[v][1] for v in chosen])
            T = np.stack([views[v][2] for v in chosen])
        K = K.astype(np.float64).copy()
        K[:, 0, :] *= w / FIX_W
        K[:, 1, :] *= h / FIX_H
        Ks.append(K)
        Rs.append(R)
        Ts.append(T)
    f = lambda a: torch.from_numpy(np.concatenate(a).astype(np.float32))
    return f(Ks), f(Rs), f(Ts)


def depth_range(batch_size, d_min=425.0, d_int=1.0, distinct=False):
    """d_min, d_int as [B,1,1,1] fp32 (the shapes the DataLoader yields, ``data.py:259-276``)."""
    if distinct:
        dm = torch.tensor([d_min + 60.0 * b for b in range(batch_size)], dtype=torch.float32)
        di = torch.tensor([d_int * (1.0 + 0.5 * b) for b in range(batch_size)], dtype=torch.float32)
    else:
        dm = torch.full((batch_size,), d_min, dtype=torch.float32)
        di = torch.full((batch_size,), d_int, dtype=torch.float32)
    return dm.reshape(-1, 1, 1, 1), di.reshape(-1, 1, 1, 1)


def features(n, c, h, w, seed):
    """N(0,1) fp32 features from ``numpy.random.default_rng(seed)`` (SURVEY §8 d)."""
    rng = np.random.default_rng(seed)
    return torch.from_numpy(rng.standard_normal((n, c, h, w), dtype=np.float32))
