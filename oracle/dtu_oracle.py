"""ORACLE (test infrastructure only -- never imported by the product path): CPU restatement of the
reference's per-sample DTU input transforms (scripts/data.py), the checker for
mvs_amd.dtu.normalize_images / threshold_depth.

* normalize: data.py:202-206 -- transforms.PILToTensor (HWC uint8 -> CHW uint8),
  ConvertImageDtype(torch.float) (``image.to(float).div(255)``, torchvision's integer->float
  rule) and Normalize(mean, std) (``tensor.sub(mean[:,None,None]).div(std[:,None,None])``), as
  torch CPU ops.  torchvision is not installed here: its published algorithm is restated.
* threshold: data.py:314-315 -- cv2.threshold(x, 0, 100000, THRESH_TOZERO) then
  cv2.threshold(x, 1000, 100000, THRESH_TOZERO_INV); OpenCV's documented rules
  (TOZERO: x > t ? x : 0; TOZERO_INV: x > t ? 0 : x).  cv2 is not installed here.
"""
import numpy as np
import torch


def normalize(rgb_hwc_u8, mean, std):
    """uint8 [..., H, W, 3] -> fp32 [..., 3, H, W]."""
    t = torch.as_tensor(rgb_hwc_u8)
    t = t.movedim(-1, -3)                                  # PILToTensor: CHW
    t = t.to(torch.float32).div(255)                       # ConvertImageDtype
    m = torch.tensor(mean, dtype=torch.float32).reshape(3, 1, 1)
    s = torch.tensor(std, dtype=torch.float32).reshape(3, 1, 1)
    return t.sub(m).div(s).contiguous()                    # Normalize


def threshold(depth, lo=0.0, hi=1000.0):
    x = np.asarray(depth, np.float32)
    x = np.where(x > np.float32(lo), x, np.float32(0))     # THRESH_TOZERO
    return np.where(x > np.float32(hi), np.float32(0), x)  # THRESH_TOZERO_INV
