"""Extract the real DTU camera geometry held in the reference's pickled DataLoader.

Source: /root/reference/scripts/test_dataloader (a ``torch.save``d DataLoader).
The file is a zip archive: ``archive/data.pkl`` (the pickle opcode stream) plus one raw
little-endian storage per tensor under ``archive/data/<key>``.

Nothing from the file is executed.  ``torch.load(..., weights_only=True)`` refuses the file
(it contains ``__main__.DtuTrainDataset`` and torchvision objects), so instead this script:

  1. walks the opcode stream with ``pickletools.genops`` -- a static disassembler that only
     parses opcodes and never constructs objects, imports modules or calls ``find_class``;
  2. pairs each sample-dict key ('K', 'R', 'T', 'd', 'd_int') with the storage key named in
     the persistent-id tuple that follows it;
  3. reads those raw float32 storages straight from the zip.

Per sample the reference dataset stores (``data.py:237-276``): K (3,3,3) at feature
resolution, R (3,3,3), T (3,3,1), d (1,1,1), d_int (1,1,1); views are the reference view
followed by ``pairs[0..1]``.

Run (survey container only; /root/reference does not exist on the GPU box):
    python tests/golden/extract_dtu_cameras.py
writes tests/golden/dtu_scan1_cameras.npz.
"""
import os
import pickletools
import re
import sys
import zipfile

import numpy as np

SRC = "/root/reference/scripts/test_dataloader"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dtu_scan1_cameras.npz")
FIELDS = ("K", "R", "T", "d", "d_int")
SHAPES = {"K": (3, 3, 3), "R": (3, 3, 3), "T": (3, 3, 1), "d": (1,), "d_int": (1,)}


def scan(pkl: bytes):
    memo = {}
    strings = []          # every string value in stream order (fresh or memo-fetched)
    samples = []
    cur = None
    field = None
    last_unicode = None
    last_was_str = None
    for op, arg, _pos in pickletools.genops(pkl):
        name = op.name
        s = None
        if name in ("BINUNICODE", "SHORT_BINUNICODE", "UNICODE", "BINUNICODE8"):
            s = arg
            last_unicode = arg
        elif name in ("BINGET", "LONG_BINGET"):
            v = memo.get(arg)
            if isinstance(v, str):
                s = v
        elif name in ("BINPUT", "LONG_BINPUT"):
            if last_was_str is not None:
                memo[arg] = last_was_str
        elif name == "MEMOIZE":
            if last_was_str is not None:
                memo[len(memo)] = last_was_str
        last_was_str = s
        if s is None:
            if name == "BINPERSID" and field is not None:
                cur[field] = last_unicode  # storage key string of the persistent id
                field = None
            continue
        strings.append(s)
        if s == "img_filenames":
            cur = {"files": []}
            samples.append(cur)
            field = None
        elif cur is not None and s in FIELDS and field is None and s not in cur:
            field = s
        elif cur is not None and s.endswith(".png"):
            cur["files"].append(s)
    return samples


def main():
    z = zipfile.ZipFile(SRC)
    samples = scan(z.read("archive/data.pkl"))
    out = {f: [] for f in FIELDS}
    files = []
    for smp in samples:
        for f in FIELDS:
            raw = z.read("archive/data/%s" % smp[f])
            arr = np.frombuffer(raw, dtype="<f4").reshape(SHAPES[f])
            out[f].append(arr)
        files.append(smp["files"])
    arrays = {f: np.stack(v).astype(np.float32) for f, v in out.items()}
    # view id = the NNN in rect_NNN_*.png (1-based in DTU file names)
    view_ids = np.array([[int(re.search(r"rect_(\d+)_", p).group(1)) for p in fl] for fl in files],
                        dtype=np.int64)
    np.savez(OUT, view_ids=view_ids, **arrays)
    print("wrote %s: %d samples, K %s, d[0]=%g d_int[0]=%g" % (
        OUT, len(samples), arrays["K"].shape, arrays["d"][0, 0], arrays["d_int"][0, 0]))


if __name__ == "__main__":
    sys.exit(main())
