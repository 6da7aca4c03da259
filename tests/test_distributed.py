"""CPU, gloo, world_size 2: the multi-GPU exchange logic of mvs_amd.depth_shards.

Each rank computes its D-slab of the cost volume (here with the oracle, on the CPU -- the HIP
kernel computes the same slab on the GPU via d_begin/d_count, see test_gpu_parity
test_depth_shards_concatenate_to_full_volume), then gather_depth_slabs reassembles the volume;
it must equal the single-process volume bit for bit, on every rank.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import sys
    for sub in ("deep-multiview-depth-estimation_amd", "oracle", os.path.join("tests", "golden")):
        sys.path.insert(0, os.path.join(REPO, sub))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(2)
        import mvs_oracle
        from cameras import camera_batch, depth_range, features
        from mvs_amd.depth_shards import gather_depth_slabs, owned_samples, plane_shard
        B, V, C, h, w, D = 3, 3, 4, 10, 14, 8
        K, R, T = camera_batch(B, V, h, w)
        d_min, d_int = depth_range(B, d_int=40.0, distinct=True)
        feat = features(B * V, C, h, w, seed=4)
        warped, _, _ = mvs_oracle.homography_warping(K, R, T, d_min, d_int, feat, B, V, D,
                                                     concat_growth=False)
        full = mvs_oracle.assemble_cost_volume(warped, V)
        begin, count = plane_shard(D, world, rank)
        slab = full[:, :, begin:begin + count].clone()
        got = gather_depth_slabs(slab, world)
        ok = torch.equal(got, full)
        mine = owned_samples(B, world, rank)
        q.put((rank, ok, mine))
    finally:
        dist.destroy_process_group()


def test_gather_depth_slabs_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [True, True]
    assert res[0][2] == [0, 2] and res[1][2] == [1]
