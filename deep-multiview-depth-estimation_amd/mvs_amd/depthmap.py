"""Drop-in for ``scripts/depthmap.py`` (``extract_depth_map``, :4-22).

Keeps the reference's permutation-indexed mask exactly: plane r is kept when the r-th entry of
``argsort(P, descending)`` is < N_DEPTH_EST (this is NOT a true top-N), ties in
P ordered by ascending plane index.  Runs in ``mvs::extract_depth_map`` (HIP): per pixel the
N_DEPTH_EST ranks are counted in one pass over D instead of sorting D values.
"""
from . import ops
from .config import N_DEPTH_EST


def extract_depth_map(prob_volume, d_batch, n_depth_est=None):
    n_est = int(N_DEPTH_EST if n_depth_est is None else n_depth_est)
    return ops.extract_depth_map_op(prob_volume, d_batch, n_est)
