"""Deterministic MVSNet weights shared by the golden-vector generator and the tests.

No state_dict ships with the fixtures: both sides regenerate the same tensors from this formula
(numpy PCG64, ``default_rng(seed)``), walking ``state_dict()`` keys in sorted order:

  * conv / deconv ``*.weight`` (4-D / 5-D): N(0,1) * sqrt(2 / fan_in), fan_in = prod(shape[1:])
    for convs; deconvs use shape[0] * prod(shape[2:]) (ConvTranspose weight is [in, out, k...]);
  * BatchNorm ``weight`` 1 + 0.1 N, ``bias`` 0.1 N, ``running_mean`` 0.1 N,
    ``running_var`` 1 + 0.1 |N|, ``num_batches_tracked`` 0.

The key set is the reference's (``scripts/model.py:155-166``: feature_encoder.model.N.*,
cost_volume_reg.conv_*/deconv_*/BN_*, depthmap_refine.model.N.*).
"""
import numpy as np
import torch


def deterministic_state_dict(state_dict, seed=1234):
    rng = np.random.default_rng(seed)
    out = {}
    for key in sorted(state_dict.keys()):
        t = state_dict[key]
        shape = tuple(t.shape)
        if key.endswith("num_batches_tracked"):
            out[key] = torch.zeros_like(t)
            continue
        if key.endswith("weight") and len(shape) >= 4:
            if "deconv" in key:
                fan_in = shape[0] * int(np.prod(shape[2:]))
            else:
                fan_in = int(np.prod(shape[1:]))
            val = rng.standard_normal(shape) * np.sqrt(2.0 / fan_in)
        elif key.endswith("running_var"):
            val = 1.0 + 0.1 * np.abs(rng.standard_normal(shape))
        elif key.endswith("running_mean") or key.endswith("bias"):
            val = 0.1 * rng.standard_normal(shape)
        elif key.endswith("weight"):
            val = 1.0 + 0.1 * rng.standard_normal(shape)
        else:
            raise KeyError("unexpected state_dict entry %s" % key)
        out[key] = torch.from_numpy(np.asarray(val, dtype=np.float32)).reshape(shape)
    return out
