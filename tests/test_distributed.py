"""CPU, gloo, world_size 2: the multi-GPU path of mvs_amd.depth_shards.

* ``exchange_to_owners`` / ``gather_depth_slabs``: each rank computes its D-slab of the cost
  volume (here with the oracle, on the CPU -- the HIP kernel computes the same slab on the GPU via
  d_begin/d_count, see test_gpu_parity test_depth_shards_concatenate_to_full_volume); the owner of
  each sample must end with exactly the single-process volume of that sample, bit for bit.
* ``DepthShardedMVSNet.forward`` end to end with the oracle injected as the slab producer and
  soft-argmin (``ops=``) and the regulariser/refinement on the CPU: every rank's owned depth maps
  must equal the single-process model's (model.py:168-207 via oracle.mvsnet_forward), and with the
  default ``gather=True`` rank 0 must hold ALL B maps (SURVEY.md §8 e step 4) equal to the
  single-process model's; B=3 (rank 0 owns samples 0 and 2, rank 1 owns sample 1) and B=1 (cfg 4's
  shape: rank 1 owns nothing).
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


def _setup(rank, world, port):
    import sys
    for sub in ("deep-multiview-depth-estimation_amd", "oracle", os.path.join("tests", "golden")):
        sys.path.insert(0, os.path.join(REPO, sub))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)


def _exchange_worker(rank, world, port, q):
    _setup(rank, world, port)
    try:
        import mvs_oracle
        from cameras import camera_batch, depth_range, features
        from mvs_amd.depth_shards import exchange_to_owners, gather_depth_slabs, owned_samples, plane_shard
        B, V, C, h, w, D = 3, 3, 4, 10, 14, 8
        K, R, T = camera_batch(B, V, h, w)
        d_min, d_int = depth_range(B, d_int=40.0, distinct=True)
        feat = features(B * V, C, h, w, seed=4)
        warped, _, _ = mvs_oracle.homography_warping(K, R, T, d_min, d_int, feat, B, V, D,
                                                     concat_growth=False)
        full = mvs_oracle.assemble_cost_volume(warped, V)
        begin, count = plane_shard(D, world, rank)
        slab = full[:, :, begin:begin + count].clone()
        mine = owned_samples(B, world, rank)
        own = exchange_to_owners(slab, world, rank)
        ok_owner = tuple(own.shape) == (len(mine), C, D, h, w) and torch.equal(own, full[mine])
        ok_all = torch.equal(gather_depth_slabs(slab, world), full)
        q.put((rank, ok_owner, ok_all, mine))
    finally:
        dist.destroy_process_group()


class _OracleOps:
    """The oracle as DepthShardedMVSNet's slab producer and soft-argmin (CPU)."""

    @staticmethod
    def cost_volume_slab(K, R, T, d_min, d_int, feats, batch_size, n_views, d_num, d_scale, d_begin,
                         d_count):
        import mvs_oracle
        warped, d_batch, ref_views = mvs_oracle.homography_warping(
            K, R, T, d_min, d_int, feats, batch_size, n_views, d_num, d_scale, concat_growth=False)
        cv = mvs_oracle.assemble_cost_volume(warped, n_views)
        return cv[:, :, d_begin:d_begin + d_count].contiguous(), d_batch, ref_views

    @staticmethod
    def extract_depth_map(prob, d_batch, n_est):
        import mvs_oracle
        return mvs_oracle.extract_depth_map(prob, d_batch, n_est)


def _model_worker(rank, world, port, B, q):
    _setup(rank, world, port)
    try:
        import mvs_oracle
        from cameras import camera_batch, depth_range
        from weights import deterministic_state_dict
        from mvs_amd.config import MVSConfig
        from mvs_amd.depth_shards import DepthShardedMVSNet
        from mvs_amd.model import MVSNet
        V, D, H, W = 3, 8, 64, 80
        net = MVSNet(MVSConfig(d_num=D, in_h=H, in_w=W), device=torch.device("cpu"))
        net.load_state_dict(deterministic_state_dict(net.state_dict()))
        net.eval()
        net.cost_volume_reg.live_region = False   # the oracle's op sequence (forward_full) on both sides
        K, R, T = camera_batch(B, V, H // 4, W // 4)
        d_min, d_int = depth_range(B, d_int=6.0, distinct=True)
        img = torch.randn(B * V, 3, H, W, generator=torch.Generator().manual_seed(11))
        sharded = DepthShardedMVSNet(net, world, rank, ops=_OracleOps, gather=False)
        with torch.no_grad():
            ini1, ref1, _ = mvs_oracle.mvsnet_forward(net, img, K, R, T, d_min, d_int, B, V, D,
                                                      (H // 4, W // 4))
            mine, ini, ref = sharded(img, K, R, T, d_min, d_int, B, V)
            # the default: every sample's maps gathered on rank 0 (MVSNet.forward's return value there)
            g_ini, g_ref = DepthShardedMVSNet(net, world, rank, ops=_OracleOps)(img, K, R, T, d_min, d_int, B, V)
        ok = True
        if mine:
            ok = (torch.allclose(ini, ini1[mine], rtol=1e-6, atol=0)
                  and torch.allclose(ref, ref1[mine], rtol=1e-5, atol=1e-3))
        else:
            ok = ini is None and ref is None
        if rank == 0:
            ok = ok and (tuple(g_ini.shape) == (B, 1, H // 4, W // 4) and torch.allclose(g_ini, ini1, rtol=1e-6, atol=0)
                         and torch.allclose(g_ref, ref1, rtol=1e-5, atol=1e-3))
            if mine:   # the gathered maps of rank 0's own samples are its own results, bit for bit
                ok = ok and torch.equal(g_ini[mine], ini) and torch.equal(g_ref[mine], ref)
        else:
            ok = ok and g_ini is None and g_ref is None
        # inference-only: autograd enabled or train-mode BN must raise, not silently diverge
        raised = 0
        try:
            sharded(img, K, R, T, d_min, d_int, B, V)
        except RuntimeError:
            raised += 1
        net.train()
        try:
            with torch.no_grad():
                sharded(img, K, R, T, d_min, d_int, B, V)
        except RuntimeError:
            raised += 1
        q.put((rank, ok, mine, raised))
    finally:
        dist.destroy_process_group()


def _run(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _opcount_worker(rank, world, port, q):
    """exchange_to_owners / gather_depth_slabs at C = 32 (the model's channel count): the number of
    point-to-point ops each posts, counted at dist.batch_isend_irecv, and the results."""
    _setup(rank, world, port)
    try:
        from mvs_amd import depth_shards
        from mvs_amd.depth_shards import exchange_plan, exchange_to_owners, gather_depth_slabs, owned_samples
        B, C, Dl, h, w = 3, 32, 4, 6, 7
        g = torch.Generator().manual_seed(0)
        full = torch.randn(B, C, world * Dl, h, w, generator=g)       # same on every rank
        slab = full[:, :, rank * Dl:(rank + 1) * Dl].clone()
        counts = []
        real = dist.batch_isend_irecv

        def counting(ops):
            counts.append(len(ops))
            return real(ops)
        depth_shards.dist.batch_isend_irecv = counting
        try:
            own = exchange_to_owners(slab, world, rank)
            every = gather_depth_slabs(slab, world)
        finally:
            depth_shards.dist.batch_isend_irecv = real
        mine = owned_samples(B, world, rank)
        q.put((rank, counts, len(exchange_plan(B, world, rank)), torch.equal(own, full[mine]),
               torch.equal(every, full)))
    finally:
        dist.destroy_process_group()


def test_exchange_posts_one_message_per_sample_and_peer():
    """At C = 32 the exchange posts one op per (sample, peer) -- 3 per rank for B = 3 on 2 ranks
    (rank 0 owns samples 0 and 2: two receives, one send) -- not one per channel (96), and the
    all-gather one send + one receive per peer; both still reassemble the volume bit for bit."""
    res = _run(_opcount_worker, 2)
    for rank, counts, planned, ok_own, ok_all in res:
        assert counts == [planned, 2] and planned == 3, (rank, counts, planned)
        assert ok_own and ok_all


def test_exchange_to_owners_world2():
    res = _run(_exchange_worker, 2)
    assert [(r[1], r[2]) for r in res] == [(True, True), (True, True)]
    assert res[0][3] == [0, 2] and res[1][3] == [1]


@pytest.mark.parametrize("B", [3, 1])
def test_depth_sharded_model_world2(B):
    res = _run(_model_worker, 2, B)
    assert all(r[1] for r in res), res
    assert res[0][2] == ([0, 2] if B == 3 else [0]) and res[1][2] == ([1] if B == 3 else [])
    assert all(r[3] == 2 for r in res), res


def _bench_dshard_worker(rank, world, port, q):
    """bench.py's own D-sharded step (bench.dshard_step) and its per-phase timing
    (bench.dshard_phase_ms), on the CPU with the oracle as the slab producer: the step must return
    every sample's maps on rank 0 equal to the single-process oracle model's, and the phase record
    must come back all-gathered, five non-negative phases per rank."""
    _setup(rank, world, port)
    try:
        import sys
        sys.path.insert(0, REPO)
        import bench
        import mvs_oracle
        from cameras import camera_batch, depth_range
        from weights import deterministic_state_dict
        from mvs_amd.config import MVSConfig
        from mvs_amd.model import MVSNet
        B, V, D, H, W = 1, 3, 8, 64, 80   # cfg 4's shape at test size: one sample, D split over the ranks
        net = MVSNet(MVSConfig(d_num=D, in_h=H, in_w=W), device=torch.device("cpu"))
        net.load_state_dict(deterministic_state_dict(net.state_dict()))
        net.eval()
        net.cost_volume_reg.live_region = False
        K, R, T = camera_batch(B, V, H // 4, W // 4)
        d_min, d_int = depth_range(B, d_int=6.0, distinct=True)
        img = torch.randn(B * V, 3, H, W, generator=torch.Generator().manual_seed(11))
        inputs = (img, K, R, T, d_min, d_int)
        sharded, step = bench.dshard_step(net, world, rank, inputs, B, V, ops=_OracleOps)
        with torch.no_grad():
            ini, ref = step()
            ini1, ref1, _ = mvs_oracle.mvsnet_forward(net, img, K, R, T, d_min, d_int, B, V, D, (H // 4, W // 4))
        phases = bench.dshard_phase_ms(sharded, step, 2, torch.device("cpu"), world)
        ok = (len(phases) == world and all(len(p) == len(bench.DSHARD_PHASES) for p in phases)
              and all(v >= 0.0 for p in phases for v in p))
        if rank == 0:
            ok = ok and torch.allclose(ini, ini1, rtol=1e-6, atol=0) and torch.allclose(ref, ref1, rtol=1e-5, atol=1e-3)
            ok = ok and phases[1][bench.DSHARD_PHASES.index("owner_compute")] < phases[0][
                bench.DSHARD_PHASES.index("owner_compute")]   # rank 1 owns no sample at B = 1
        else:
            ok = ok and ini is None and ref is None
        q.put((rank, ok, phases))
    finally:
        dist.destroy_process_group()


def test_bench_dshard_step_world2():
    """The D-sharded step exactly as bench.py --mode dshard builds and times it (gloo, world 2, CPU)."""
    res = _run(_bench_dshard_worker, 2)
    assert all(r[1] for r in res), res
    assert res[0][2] == res[1][2]   # the all-gathered phase table is the same on both ranks
