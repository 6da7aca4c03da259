"""DTU readers and input transforms (reference scripts/data.py).

CPU tests pin the host readers: cam.txt / pair.txt / PFM parsing and the sample assembly
(data.py:18-80, 237-276, 327-358) against the real DTU scan-1 cameras the reference's own pickled
test DataLoader holds (tests/golden/dtu_scan1_cameras.npz: K/R/T/d/d_int and the (ref, pair0, pair1)
view ids of all 49 samples).  The on-disk tree is synthesised from those values (the DTU files
themselves are not in the reference).  GPU tests check the HIP transforms bit-exactly against the
oracle (oracle/dtu_oracle.py).  Image pixels are synthetic: no DTU image ships with the reference.
"""
import os

import numpy as np
import pytest
import torch

import dtu_oracle
from cameras import load_fixture
from mvs_amd import dtu


def _write_cam(path, K, R, T, d, d_int):
    with open(path, "w") as f:
        f.write("extrinsic\n")
        for r in range(3):
            f.write(" ".join(repr(float(x)) for x in list(R[r]) + [T[r, 0]]) + "\n")
        f.write("0.0 0.0 0.0 1.0\n\nintrinsic\n")
        for r in range(3):
            f.write(" ".join(repr(float(x)) for x in K[r]) + "\n")
        f.write("\n%r %r\n" % (float(d), float(d_int)))


def _make_tree(root, n_img_hw=(16, 20), depth_hw=(4, 5), with_images=True):
    """DTU layout (data.py:26-36, 91-96, 148-160) with the fixture's 49 scan-1 cameras."""
    fx = load_fixture()
    cam_dir = os.path.join(root, "Cameras", "train")
    os.makedirs(cam_dir, exist_ok=True)
    # view id v (1..49) <-> camera index v-1; every sample's reference view appears once
    refs = {int(fx["view_ids"][s, 0]) - 1: s for s in range(49)}
    for cam, s in refs.items():
        _write_cam(os.path.join(cam_dir, "%08d_cam.txt" % cam), fx["K"][s, 0], fx["R"][s, 0],
                   fx["T"][s, 0], fx["d"][s, 0], fx["d_int"][s, 0])
    with open(os.path.join(root, "Cameras", "pair.txt"), "w") as f:
        f.write("49\n")
        for cam in range(49):
            s = refs[cam]
            src = [int(v) - 1 for v in fx["view_ids"][s, 1:]]
            src += [c for c in range(49) if c != cam and c not in src][:8]
            f.write("%d\n10 %s\n" % (cam, " ".join("%d %.2f" % (c, 100.0 - i) for i, c in enumerate(src))))
    rng = np.random.default_rng(11)
    img_dir = os.path.join(root, "Rectified", "scan1_train")
    dep_dir = os.path.join(root, "Depths", "scan1_train")
    os.makedirs(img_dir, exist_ok=True)
    os.makedirs(dep_dir, exist_ok=True)
    if with_images:
        from PIL import Image
        for cam in range(49):
            Image.fromarray(rng.integers(0, 256, n_img_hw + (3,), dtype=np.uint8)).save(
                os.path.join(img_dir, "rect_%03d_0_r5000.png" % (cam + 1)))
            dep = rng.uniform(-200, 1400, depth_hw).astype(np.float32)
            dtu.write_pfm(os.path.join(dep_dir, "depth_map_%04d.pfm" % cam), dep)
    return fx, refs


def test_cam_and_pair_readers_reproduce_reference_cameras(tmp_path):
    fx, refs = _make_tree(str(tmp_path), with_images=False)
    cams = dtu.Cameras(str(tmp_path), np.arange(49))
    for cam, s in refs.items():
        assert np.array_equal(np.float32(cams.K[cam]), fx["K"][s, 0])
        assert np.array_equal(np.float32(cams.R[cam]), fx["R"][s, 0])
        assert np.array_equal(np.float32(cams.T[cam]), fx["T"][s, 0])
        assert cams.d[cam].shape == (1, 1) and np.float32(cams.d[cam][0, 0]) == fx["d"][s, 0]
        assert np.float32(cams.d_int[cam][0, 0]) == fx["d_int"][s, 0]
        assert list(cams.pairs[cam][:2]) == [int(v) - 1 for v in fx["view_ids"][s, 1:]]
        assert len(cams.pairs[cam]) == 10


def test_pair_reader_keeps_first_line_character_quirk(tmp_path):
    """data.py:74-76: the first id line is tested by its first CHARACTER ('12' -> 1)."""
    p = tmp_path / "pair.txt"
    p.write_text("2\n12\n2 3 1.0 4 2.0\n13\n2 5 1.0 6 2.0\n")
    assert [list(x) for x in dtu.read_pair_file(str(p), [1])] == [[3, 4]]
    assert [list(x) for x in dtu.read_pair_file(str(p), [1, 13])] == [[3, 4], [5, 6]]


@pytest.mark.parametrize("scale", [1.0, -1.0])
def test_pfm_roundtrip_and_flip(tmp_path, scale):
    a = np.arange(12, dtype=np.float32).reshape(3, 4) * 1.5
    p = str(tmp_path / "d.pfm")
    dtu.write_pfm(p, a, scale=scale)
    assert np.array_equal(dtu.load_depth(p), a)
    raw = np.frombuffer(open(p, "rb").read().split(b"\n", 3)[3], "<f" if scale > 0 else ">f")
    assert np.array_equal(raw.reshape(3, 4), a[::-1])   # stored bottom-up, data.py:357 flips


def test_pfm_rejects_bad_header(tmp_path):
    p = tmp_path / "bad.pfm"
    p.write_bytes(b"PX\n1 1 \n1.0\n\x00\x00\x00\x00")
    with pytest.raises(Exception, match="Invalid Header"):
        dtu.load_depth(str(p))


def test_dataset_assembles_reference_triples(tmp_path):
    fx, refs = _make_tree(str(tmp_path), with_images=False)
    reader = dtu.DtuReader(str(tmp_path), np.arange(49), np.array([1]), "test")
    ds = dtu.DtuTrainDataset(reader, device="cpu", raw=True)
    assert len(ds) == 49
    for cam, s in refs.items():
        smp = ds.samples[cam]
        ids = [int(v) for v in fx["view_ids"][s]]
        assert [os.path.basename(p) for p in smp["img_filenames"]] == \
            ["rect_%03d_0_r5000.png" % v for v in ids]
        assert smp["K"].shape == (3, 3, 3) and smp["T"].shape == (3, 3, 1)
        assert smp["d"].shape == (1, 1, 1) and smp["d_int"].shape == (1, 1, 1)
        assert np.array_equal(smp["K"].numpy(), fx["K"][s])
        assert np.array_equal(smp["R"].numpy(), fx["R"][s])
        assert np.array_equal(smp["T"].numpy(), fx["T"][s])


def test_transforms_refuse_cpu_tensors():
    from mvs_amd._lib import MVSLibraryError
    with pytest.raises(MVSLibraryError):
        dtu.normalize_images(torch.zeros(1, 2, 2, 3, dtype=torch.uint8))
    with pytest.raises(MVSLibraryError):
        dtu.threshold_depth(torch.zeros(4))


@pytest.mark.gpu
@pytest.mark.parametrize("hw", [(512, 640), (7, 9), (1, 1)])
def test_normalize_images_bit_exact(hw):
    rng = np.random.default_rng(hw[0])
    rgb = rng.integers(0, 256, (3,) + hw + (3,), dtype=np.uint8)
    rgb[0, 0, 0] = [0, 255, 128]
    out = dtu.normalize_images(torch.from_numpy(rgb).cuda()).cpu()
    ref = dtu_oracle.normalize(rgb, dtu.DTU_MEAN, dtu.DTU_STD)
    assert out.shape == ref.shape and torch.equal(out, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [128 * 160, 4 * 5, 3])
def test_depth_threshold_bit_exact(n):
    rng = np.random.default_rng(n)
    x = rng.uniform(-500, 1500, n).astype(np.float32)
    x[: min(n, 3)] = [0.0, 1000.0, np.nan][: min(n, 3)]
    out = dtu.threshold_depth(torch.from_numpy(x).cuda()).cpu().numpy()
    assert np.array_equal(out, dtu_oracle.threshold(x), equal_nan=False)


@pytest.mark.gpu
def test_dataset_item_and_batch_match_oracle(tmp_path):
    _make_tree(str(tmp_path))
    reader = dtu.DtuReader(str(tmp_path), np.arange(49), np.array([1]), "test")
    ds = dtu.DtuTrainDataset(reader, device="cuda:0")
    raw = dtu.DtuTrainDataset(reader, device="cuda:0", raw=True)
    item = ds[5]
    r = raw.raw_item(5)
    assert item["input_img"].shape == (3, 3, 16, 20) and item["depth_ref"].shape == (1, 1, 4, 5)
    assert torch.equal(item["input_img"].cpu(), dtu_oracle.normalize(r["rgb"].numpy(), dtu.DTU_MEAN, dtu.DTU_STD))
    assert np.array_equal(item["depth_ref"].cpu().numpy()[0, 0], dtu_oracle.threshold(r["depth_raw"].numpy()))
    batch = dtu.collate_to_device([raw[i] for i in (5, 9)], "cuda:0")
    assert batch["input_img"].shape == (2, 3, 3, 16, 20) and batch["depth_ref"].shape == (2, 1, 1, 4, 5)
    assert torch.equal(batch["input_img"][0].cpu(), item["input_img"].cpu())
    assert batch["K"].shape == (2, 3, 3, 3) and batch["d"].shape == (2, 1, 1, 1)
