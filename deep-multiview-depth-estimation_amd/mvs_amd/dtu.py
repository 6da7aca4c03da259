"""DTU on-disk readers and the per-batch input transforms: drop-in for
``scripts/data.py`` (``Cameras``, ``Depths``, ``Rectified``, ``DtuReader``, ``DtuTrainDataset``,
``load_depth``, ``get_dtu_loader``).

File parsing stays on the host (text cam/pair files, PFM, PNG decode through PIL, as the
reference does); the two per-sample tensor transforms run on the GPU through the C ABI:

* ``normalize_images``  -- data.py:202-206 + 306-311 (PILToTensor -> ConvertImageDtype(float) ->
  Normalize(mean, std)) as ``mvs_normalize_images``: uint8 HWC in, fp32 NCHW out, bit-identical
  to torch's CPU ops.  Only the decoded uint8 pixels cross PCIe (1/4 of the fp32 bytes).
* ``threshold_depth``   -- data.py:314-315 (cv2 THRESH_TOZERO at 0, THRESH_TOZERO_INV at 1000) as
  ``mvs_depth_threshold``.

``DtuTrainDataset`` therefore yields what the reference's yields (same dict keys, shapes and
dtypes: ``input_img`` [V,3,H,W] fp32, ``depth_ref`` [1,1,H,W], K/R/T [V,3,3]/[V,3,3]/[V,3,1], d and
d_int [1,1,1]) when ``device`` is a GPU; ``collate_to_device`` batches raw samples and runs the
transforms once per batch on the GPU instead (the faster path for ``train.py``-style loops).
There is no CPU fallback for the transforms: a CPU ``device`` raises ``MVSLibraryError``.
"""
import ctypes
import re
from itertools import product
from os.path import join

import numpy as np
import torch

from . import _lib

# data.py:198-199 (precomputed over the DTU training images)
DTU_MEAN = (0.3941, 0.3366, 0.2942)
DTU_STD = (0.3387, 0.3264, 0.3185)
DEPTH_LO, DEPTH_HI = 0.0, 1000.0   # data.py:314-315


# ----------------------------------------------------------------------------------------------
# text formats
# ----------------------------------------------------------------------------------------------
def read_cam_file(path):
    """One ``<id>_cam.txt`` (data.py:40-68): returns K [3,3], R [3,3], T [3,1], d [1,1], d_int [1,1]
    as float64 arrays.  Layout: a text line, 4 extrinsic rows [R|T], two skipped lines, 3
    intrinsic rows, a skipped line, then ``d_min d_interval``."""
    with open(path) as f:
        f.readline()
        ext = [np.float64(f.readline().split()) for _ in range(4)]
        f.readline()
        f.readline()
        intr = [np.float64(f.readline().split()) for _ in range(3)]
        f.readline()
        dline = np.float64(f.readline().split())
    K = np.vstack(intr)
    R = np.vstack([e[0:3] for e in ext[:3]])
    T = np.vstack([e[-1] for e in ext[:3]])
    return K, R, T, np.array([dline[0]]).reshape(-1, 1), np.array([dline[1]]).reshape(-1, 1)


def read_pair_file(path, cam_list):
    """``pair.txt`` (data.py:70-80): for every listed reference view, its source-view ids.

    Keeps the reference's parse exactly, including its quirk: the FIRST reference-id line is
    tested by its first character (``int(line[0])`` of a string), later ones by their first
    token; a reference whose id is not in ``cam_list`` leaves its pair line to be read as the next
    id line (the count field then acts as an id)."""
    cams = set(int(c) for c in cam_list)
    pairs = []
    with open(path) as f:
        f.readline()
        line = f.readline()
        while line:
            if int(line[0]) in cams:
                pair_line = f.readline().split()
                pairs.append(np.int64(pair_line[1::2]))
            line = f.readline().split()
    return pairs


def load_depth(path):
    """PFM reader (data.py:327-358): float32 [H, W, C] flipped vertically (cv2.flip(data, 0))."""
    with open(path, "rb") as f:
        header = f.readline().decode("UTF-8").rstrip()
        dim_match = re.match(r"^(\d+)\s(\d+)\s$", f.readline().decode("UTF-8"))
        scale = float(f.readline().decode("UTF-8").rstrip())
        data = f.read()
    if header == "PF":
        ch = 3
    elif header == "Pf":
        ch = 1
    else:
        raise Exception("Invalid Header for PFM file.")
    if not dim_match:
        raise Exception("PFM header gives no dimensions.")
    width, height = map(int, dim_match.groups())
    arr = np.frombuffer(data, "<f" if scale > 0 else ">f").reshape(height, width, ch)
    # cv2.flip returns a native-endian float32 copy; the single-channel case drops the channel
    # axis (cv2 arrays are 2-D for 1 channel)
    out = np.ascontiguousarray(arr[::-1]).astype(np.float32)
    return out[:, :, 0] if ch == 1 else out


def write_pfm(path, data, scale=1.0):
    """Writer for the format ``load_depth`` reads (used by the tests' fixtures)."""
    data = np.asarray(data, np.float32)
    ch = 3 if data.ndim == 3 and data.shape[2] == 3 else 1
    h, w = data.shape[:2]
    with open(path, "wb") as f:
        f.write(("PF\n" if ch == 3 else "Pf\n").encode())
        f.write(("%d %d \n" % (w, h)).encode())   # data.py:332 requires '<w> <h> ' + newline
        f.write(("%f\n" % (-abs(scale) if scale < 0 else abs(scale))).encode())
        arr = np.ascontiguousarray(data.reshape(h, w, ch)[::-1])
        f.write(arr.astype("<f" if scale > 0 else ">f").tobytes())


# ----------------------------------------------------------------------------------------------
# GPU transforms (C ABI)
# ----------------------------------------------------------------------------------------------
def normalize_images(rgb, mean=DTU_MEAN, std=DTU_STD):
    """uint8 [N, H, W, 3] (GPU) -> fp32 [N, 3, H, W] normalised (data.py:202-206)."""
    if not rgb.is_cuda:
        raise _lib.MVSLibraryError("normalize_images needs a GPU tensor (no CPU fallback)")
    if rgb.dtype != torch.uint8 or rgb.dim() != 4 or rgb.shape[3] != 3:
        raise ValueError("rgb must be uint8 [N, H, W, 3], got %s %s" % (rgb.dtype, tuple(rgb.shape)))
    lib = _lib.load()
    rgb = rgb.contiguous()
    n, h, w, _ = rgb.shape
    out = torch.empty((n, 3, h, w), device=rgb.device, dtype=torch.float32)
    if n == 0:
        return out
    m = (ctypes_float3(mean), ctypes_float3(std))   # host arrays, alive across the call
    st = lib.mvs_normalize_images(_lib.ptr(rgb), n, h, w, ctypes.cast(m[0], ctypes.c_void_p),
                                  ctypes.cast(m[1], ctypes.c_void_p), _lib.ptr(out),
                                  _lib.stream_handle(rgb.device))
    _lib.check(st, "mvs_normalize_images")
    return out


def threshold_depth(depth, lo=DEPTH_LO, hi=DEPTH_HI):
    """cv2 THRESH_TOZERO at ``lo`` then THRESH_TOZERO_INV at ``hi`` (data.py:314-315), on the GPU."""
    if not depth.is_cuda:
        raise _lib.MVSLibraryError("threshold_depth needs a GPU tensor (no CPU fallback)")
    lib = _lib.load()
    src = depth.to(torch.float32).contiguous()
    out = torch.empty_like(src)
    st = lib.mvs_depth_threshold(_lib.ptr(src), src.numel(), float(lo), float(hi), _lib.ptr(out),
                                 _lib.stream_handle(src.device))
    _lib.check(st, "mvs_depth_threshold")
    return out


def ctypes_float3(v):
    return (ctypes.c_float * 3)(*[float(x) for x in v])


def decode_rgb(path):
    """PNG -> uint8 [H, W, 3] (``Image.open(..).convert('RGB')`` as data.py:306-311 does)."""
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"), dtype=np.uint8)


# ----------------------------------------------------------------------------------------------
# readers (data.py:18-183), same attributes and file-name rules
# ----------------------------------------------------------------------------------------------
class Cameras:
    """data.py:18-80: K/R/T/d/d_int lists indexed like ``cam_list`` plus ``pairs``."""

    def __init__(self, path, cam_list):
        self.cam_list = cam_list
        self.base_path = path
        self.class_path = join(path, "Cameras", "train")
        self.file_names = [join(self.class_path, "{:0>8}".format(str(i)) + "_cam.txt") for i in cam_list]
        self.K, self.R, self.T, self.d, self.d_int = [], [], [], [], []
        for fn in self.file_names:
            K, R, T, d, di = read_cam_file(fn)
            self.K.append(K)
            self.R.append(R)
            self.T.append(T)
            self.d.append(d)
            self.d_int.append(di)
        self.pairs = read_pair_file(join(self.class_path, "..", "pair.txt"), cam_list)


class Depths:
    """data.py:82-100: ``Depths/scan<k>_train/depth_map_<id:04>.pfm`` per scan and camera."""

    def __init__(self, path, cam_list, scan_idx=(1,), event="train"):
        self.cam_list = cam_list
        self.base_path = path
        self.class_path = join(path, "Depths")
        self.scan_path = [join(self.class_path, "scan" + str(s) + "_train") for s in scan_idx]
        self.file_names = [[join(sp, "depth_map_" + "{:0>4}".format(str(i)) + ".pfm") for i in cam_list]
                           for sp in self.scan_path]


class Rectified:
    """data.py:140-164: ``Rectified/scan<k>_train/rect_<id+1:03>_<light>_r5000.png``."""

    def __init__(self, path, cam_list, scan_idx=(1,), event="train"):
        self.cam_list = cam_list
        self.base_path = path
        self.class_path = join(path, "Rectified")
        self.scan_path = [join(self.class_path, "scan" + str(s) + "_train") for s in scan_idx]
        self.file_names = [[[join(sp, "rect_" + "{:0>3}".format(str(i + 1)) + "_" + str(l) + "_r5000.png")
                             for i in cam_list] for l in range(7)] for sp in self.scan_path]


class DtuReader:
    """data.py:166-183."""

    def __init__(self, folder_path, cam_idx, scan_idx, event):
        self.cam_idx = cam_idx
        self.scan_idx = scan_idx
        self.event = event
        self.Cameras = Cameras(folder_path, cam_idx)
        self.Depths = Depths(folder_path, cam_idx, scan_idx=scan_idx, event=event)
        self.Images = Rectified(folder_path, cam_idx, scan_idx=scan_idx, event=event)
        self.n_images = len(cam_idx) * len(scan_idx)

    def __len__(self):
        return self.n_images


class DtuTrainDataset(torch.utils.data.Dataset):
    """data.py:186-320: one sample per (scan, reference camera) at lighting 0, views
    [ref, pairs[ref][0], pairs[ref][1]].

    ``device`` (a GPU) is where ``__getitem__`` runs the image/depth transforms; with
    ``raw=True`` samples carry the decoded uint8 images and the unclamped depth instead, for
    ``collate_to_device`` to transform a whole batch at once."""

    def __init__(self, DTU, device=None, raw=False, mean=DTU_MEAN, std=DTU_STD):
        self.device = torch.device(device) if device is not None else torch.device("cuda", 0)
        self.raw = raw
        self.mean, self.std = mean, std
        f32 = lambda a: torch.from_numpy(np.asarray(a, np.float32)).unsqueeze(0)   # unsqz(.., 1)
        self.samples = []
        for scan, light, ref in product(range(len(DTU.scan_idx)), range(1), range(len(DTU.cam_idx))):
            p1, p2 = DTU.Cameras.pairs[ref][0], DTU.Cameras.pairs[ref][1]
            imgs = DTU.Images.file_names[scan][light]
            C = DTU.Cameras
            self.samples.append({
                "img_filenames": [imgs[ref], imgs[p1], imgs[p2]],
                "depth_filename": DTU.Depths.file_names[scan][ref],
                "K": torch.cat((f32(C.K[ref]), f32(C.K[p1]), f32(C.K[p2])), 0),
                "R": torch.cat((f32(C.R[ref]), f32(C.R[p1]), f32(C.R[p2])), 0),
                "T": torch.cat((f32(C.T[ref]), f32(C.T[p1]), f32(C.T[p2])), 0),
                "d": f32(C.d[ref]),
                "d_int": f32(C.d_int[ref]),
            })

    def __len__(self):
        return len(self.samples)

    def raw_item(self, idx):
        s = self.samples[idx]
        rgb = np.stack([decode_rgb(p) for p in s["img_filenames"]])
        depth = load_depth(s["depth_filename"])
        return {"rgb": torch.from_numpy(rgb), "depth_raw": torch.from_numpy(depth.copy()),
                "K": s["K"], "R": s["R"], "T": s["T"], "d": s["d"], "d_int": s["d_int"]}

    def __getitem__(self, idx):
        item = self.raw_item(idx)
        if self.raw:
            return item
        return _transform(item["rgb"].unsqueeze(0), item["depth_raw"].unsqueeze(0), item,
                          self.device, self.mean, self.std, batched=False)


def _transform(rgb, depth, item, device, mean, std, batched):
    """rgb [B,V,H,W,3] uint8, depth [B,H,W] -> the reference's sample/batch dict on ``device``."""
    b, v, h, w, _ = rgb.shape
    x = normalize_images(rgb.reshape(b * v, h, w, 3).to(device, non_blocking=True), mean, std)
    dep = threshold_depth(depth.to(device, non_blocking=True))
    dh, dw = dep.shape[-2], dep.shape[-1]
    if batched:
        return {"input_img": x.reshape(b, v, 3, h, w), "depth_ref": dep.reshape(b, 1, 1, dh, dw),
                "K": item["K"], "R": item["R"], "T": item["T"], "d": item["d"], "d_int": item["d_int"]}
    return {"input_img": x.reshape(v, 3, h, w), "depth_ref": dep.reshape(1, 1, dh, dw),
            "K": item["K"], "R": item["R"], "T": item["T"], "d": item["d"], "d_int": item["d_int"]}


def collate_to_device(items, device=None, mean=DTU_MEAN, std=DTU_STD):
    """Batch raw samples (``DtuTrainDataset(raw=True)``) and transform them on the GPU in one
    launch each; yields the batch dict ``train.py:86-96`` consumes (input_img [B,V,3,H,W], ...)."""
    device = torch.device(device) if device is not None else torch.device("cuda", 0)
    rgb = torch.stack([it["rgb"] for it in items])
    depth = torch.stack([it["depth_raw"] for it in items])
    if rgb.device.type == "cpu" and torch.cuda.is_available():
        rgb = rgb.pin_memory()
    cat = lambda k: torch.stack([it[k] for it in items])
    meta = {k: cat(k) for k in ("K", "R", "T", "d", "d_int")}
    return _transform(rgb, depth, meta, device, mean, std, batched=True)


def get_dtu_loader(folder_path, cam_idx, scan_idx, event, batch_size=14, i_start=0, device=None):
    """data.py:360-382 (shuffled DataLoader over DtuTrainDataset); batches are transformed on the GPU."""
    ds = DtuTrainDataset(DtuReader(folder_path, cam_idx, scan_idx, event), device=device, raw=True)
    return torch.utils.data.DataLoader(ds, batch_size=batch_size, shuffle=True,
                                       collate_fn=lambda items: collate_to_device(items, device))
