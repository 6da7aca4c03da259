"""Hot-path parameters (reference: ``scripts/config.py:4-24``).

The reference binds these as import-time module globals (``from config import D_NUM, ...``).
The same names exist here with the same default values, so ``from mvs_amd.config import *``
is a drop-in; ``MVSConfig`` carries them explicitly for callers that need several geometries
in one process (the reference cannot: it must be re-imported per geometry).
"""
import os
from dataclasses import dataclass, field

import numpy as np
import torch

ACC_THRESH = 0.05            # config.py:4
D_SCALE = 25                 # config.py:6  -- plane spacing multiplier of d_int
D_NUM = 20                   # config.py:7  -- default number of depth planes
N_DEPTH_EST = torch.tensor(5)  # config.py:9 -- soft-argmin mask size
DIM_REDUCE = 4               # config.py:12
IN_H = 512                   # config.py:13
IN_W = 640                   # config.py:14
FEAT_H = int(IN_H / DIM_REDUCE)   # config.py:16
FEAT_W = int(IN_W / DIM_REDUCE)   # config.py:17


def pad_outpad(d_num, feat_h, feat_w):
    """config.py:20-21: PAD = dim//2 + 1, OUTPAD = (dim + 1) % 2 over (D, H, W)."""
    dims = np.array([d_num, feat_h, feat_w])
    pad = tuple(int(x) for x in np.int64(np.floor(dims / 2) + 1))
    outpad = tuple(int(x) for x in (dims + 1) % 2)
    return pad, outpad


PAD, OUTPAD = pad_outpad(D_NUM, FEAT_H, FEAT_W)
DEVICE = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")  # config.py:24
ARITHMETICS = ("fp32", "split_f16")


@dataclass
class MVSConfig:
    """Explicit, per-model copy of the reference's import-time constants."""
    d_num: int = D_NUM
    d_scale: float = D_SCALE
    n_depth_est: int = 5
    in_h: int = IN_H
    in_w: int = IN_W
    dim_reduce: int = DIM_REDUCE
    feat_h: int = field(default=None)
    feat_w: int = field(default=None)
    # opt-in reduced precision: "bfloat16" stores the cost volume in bf16 (the
    # fused kernel rounds each fp32 variance once; half the HBM bytes written and read) and the 3-D
    # regulariser computes in fp32 from the rounded values; the default "float32" is the reference's
    # numerics
    cv_dtype: str = "float32"
    # the arithmetic of the HIP inference kernels.  "fp32" (default, the reference's model.py:35-59,
    # 76-89, 134-145 nn.Conv2d / Conv3d / ConvTranspose3d numerics): every product and sum in exact
    # fp32 -- VALU kernels, fp32-input MFMA (v_mfma_f32_16x16x4_f32, an fmaf chain bit for bit) and
    # the fp32 cost volume.  "split_f16" (opt-in, narrower than fp32): the encoder / refinement /
    # regulariser convolutions on the f16 matrix cores with split-fp16 operands (hi + lo fp16 parts
    # of a power-of-two-scaled fp32 value: 22 significant bits per operand, an absolute floor below
    # ~1e-5 of a tensor's bound) and the cost volume stored as those parts.
    # MVS_ARITHMETIC overrides the default for a process.
    arithmetic: str = field(default=None)

    def __post_init__(self):
        if self.arithmetic is None:
            self.arithmetic = os.environ.get("MVS_ARITHMETIC", "fp32")
        if self.arithmetic not in ARITHMETICS:
            raise ValueError("arithmetic must be one of %s, got %r" % (ARITHMETICS, self.arithmetic))
        if self.feat_h is None:
            self.feat_h = int(self.in_h / self.dim_reduce)
        if self.feat_w is None:
            self.feat_w = int(self.in_w / self.dim_reduce)

    @property
    def pad(self):
        return pad_outpad(self.d_num, self.feat_h, self.feat_w)[0]

    @property
    def outpad(self):
        return pad_outpad(self.d_num, self.feat_h, self.feat_w)[1]
