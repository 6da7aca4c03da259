"""Depth-plane sharding of the cost volume across the GPUs of one node (BASELINE configs[3]).

The fused warp+variance is independent per (sample, plane, pixel), so rank r of P computes planes
[r*D/P, (r+1)*D/P) with no communication (the kernel's ``d_begin``/``d_count``), from replicated
features and cameras.  The 3-D regulariser is NOT D-local (stride-2 convs with padding D/2+1 remap
planes non-locally, softmax and the soft-argmin span all D; SURVEY.md §8 e), so each sample's
full-D cost volume is assembled on the ONE rank that owns it (sample b -> rank b mod P), which then
runs the regulariser, soft-argmin and refinement for it:

  * owner-targeted exchange (``exchange_to_owners``): every rank sends its slab of sample b only
    to b's owner -- a gather to the owner when B < P (cfg 4: B = 1, only rank 0 receives), an
    all-to-all by sample when B >= P; nothing goes to ranks that would discard it;
  * ONE message per (sample, peer): a source rank sends its whole [C, D/P, h, w] slab of the
    sample (contiguous) and the owner receives it into a staging buffer [P, C, D/P, h, w]; one
    strided device copy then interleaves the P slabs into the final [C, D, h, w] layout (the
    regulariser's NCDHW input, where a slab is C separate blocks).  All messages of a step are one
    grouped ``batch_isend_irecv`` (RCCL over xGMI when the process group is ``nccl``): at cfg 4
    (B = 1, P = 8) rank 0 posts 7 receives of 84 MB instead of 7 x 32 per-channel ones;
  * the depth maps come back to ONE rank (``gather_depth_maps``, SURVEY.md §8 e step 4): every owner
    sends its samples' initial and refined maps as one [n_owned, 2, h, w] message to rank ``dst``,
    which returns the whole batch in sample order -- ``DepthShardedMVSNet.forward`` then has
    MVSNet.forward's return value on that rank.

Expected cfg 4 step (B = 1, D = 256, 8 ranks): each rank's 32-plane shard kernel
~0.05 ms, the exchange ~0.55 ms (the owner receives 7 x 84 MB, one slab per xGMI link in
parallel: 84 MB / 153 GB/s), the interleaving copy ~0.15 ms (671 MB read + written),
then the owner's D = 256 regulariser ~2 ms -- the other 7 GPUs idle through it, so at B = 1 the
D-sharded job is no faster than one GPU computing the whole volume: the cost volume is ~7 % of the
step, the regulariser (which cannot be D-sharded exactly) the rest.

Eval-mode inference only: BatchNorm in train mode would normalise with the statistics of the
owned samples instead of the whole batch (model.py:184), and the point-to-point exchange carries
no gradient -- ``DepthShardedMVSNet.forward`` raises in either case.

Reference: there is no multi-GPU path in the reference (single device, ``config.py:24``); this
module reproduces ``model.py:168-207`` for every owned sample.
"""
import torch
import torch.distributed as dist
import torch.nn as nn


def plane_shard(d_num, world, rank):
    """[begin, count) of the planes rank ``rank`` computes; D must split evenly."""
    if d_num % world:
        raise ValueError("d_num=%d does not split over %d ranks" % (d_num, world))
    count = d_num // world
    return rank * count, count


def owned_samples(batch_size, world, rank):
    """Samples whose regulariser/soft-argmin this rank runs (round-robin)."""
    return [b for b in range(batch_size) if b % world == rank]


def exchange_plan(batch_size, world, rank):
    """The point-to-point messages of exchange_to_owners on this rank: a list of
    ("send" | "recv", peer, sample), one per (sample, peer) pair that must move -- a sample's slab
    goes from every non-owner rank to its owner and nowhere else."""
    plan = []
    for b in range(batch_size):
        owner = b % world
        if owner != rank:
            plan.append(("send", owner, b))
        else:
            plan += [("recv", src, b) for src in range(world) if src != rank]
    return plan


def exchange_to_owners(slab, world, rank, group=None):
    """Owner-targeted exchange of cost-volume D-slabs.

    ``slab`` is this rank's [B, C, Dl, h, w] (planes [rank*Dl, (rank+1)*Dl) of every sample).
    Returns the full-D volume [len(owned_samples), C, world*Dl, h, w] of the samples this rank
    owns (an empty tensor when it owns none).  Every rank must call it (collective).  One message
    per (sample, peer) (``exchange_plan``), received into a per-sample staging buffer and
    interleaved into the NCDHW result by one strided copy per owned sample."""
    slab = slab.contiguous()
    b_all, c, dl, h, w = slab.shape
    mine = owned_samples(b_all, world, rank)
    out = slab.new_empty((len(mine), c, world * dl, h, w))
    if world == 1:
        for i, b in enumerate(mine):
            out[i].copy_(slab[b])
        return out
    stage = {b: slab.new_empty((world, c, dl, h, w)) for b in mine}
    ops = []
    for kind, peer, b in exchange_plan(b_all, world, rank):
        if kind == "send":
            ops.append(dist.P2POp(dist.isend, slab[b], peer, group))
        else:
            ops.append(dist.P2POp(dist.irecv, stage[b][peer], peer, group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    for i, b in enumerate(mine):
        stage[b][rank].copy_(slab[b])
        interleave_slabs(stage[b], out[i])
    return out


def interleave_slabs(stage, out):
    """The owner's interleave: ``stage`` [P, C, Dl, h, w] (slab p = planes [p Dl, (p + 1) Dl) of every
    channel, as received) -> ``out`` [C, P Dl, h, w] (NCDHW), one strided device copy."""
    p, c, dl, h, w = stage.shape
    out.view(c, p, dl, h, w).copy_(stage.transpose(0, 1))
    return out


def gather_depth_slabs(slab, world, group=None):
    """All-gather [B, C, Dl, h, w] slabs (rank order = plane order) into [B, C, world*Dl, h, w] on
    every rank (every rank then holds every sample: use exchange_to_owners when only the owner
    needs a sample's volume).  One message per peer (the whole contiguous slab), staged and
    interleaved by one strided copy."""
    if world == 1:
        return slab
    slab = slab.contiguous()
    b, c, dl, h, w = slab.shape
    rank = dist.get_rank(group)
    stage = slab.new_empty((world, b, c, dl, h, w))
    ops = []
    for peer in range(world):
        if peer != rank:
            ops.append(dist.P2POp(dist.isend, slab, peer, group))
            ops.append(dist.P2POp(dist.irecv, stage[peer], peer, group))
    for req in dist.batch_isend_irecv(ops):
        req.wait()
    stage[rank].copy_(slab)
    out = slab.new_empty((b, c, world * dl, h, w))
    out.view(b, c, world, dl, h, w).copy_(stage.permute(1, 2, 0, 3, 4, 5))
    return out


def gather_depth_maps(initial, refined, batch_size, world, rank, h, w, dst=0, group=None, device=None,
                      dtype=torch.float32):
    """The owners' depth maps -> rank ``dst`` in sample order (SURVEY.md §8 e step 4).

    ``initial`` / ``refined``: this rank's owned samples' maps [len(owned_samples), 1, h, w] (None
    when it owns none).  Every rank must call it.  Each owner other than ``dst`` sends ONE message
    ([n_owned, 2, h, w]: initial and refined stacked, 160 KB per sample at 128 x 160); ``dst`` posts
    one receive per such peer, sized from owned_samples.  Returns (initial [B, 1, h, w], refined
    [B, 1, h, w]) on ``dst``, (None, None) elsewhere."""
    mine = owned_samples(batch_size, world, rank)
    pack = None if not mine else torch.cat((initial, refined), dim=1).contiguous()
    if rank != dst:
        if mine and world > 1:
            for req in dist.batch_isend_irecv([dist.P2POp(dist.isend, pack, dst, group)]):
                req.wait()
        return None, None
    dev, dt = (pack.device, pack.dtype) if pack is not None else (device, dtype)
    out = torch.empty((batch_size, 2, h, w), device=dev, dtype=dt)
    ops, recvd = [], []
    for src in range(world):
        own = owned_samples(batch_size, world, src)
        if not own:
            continue
        if src == rank:
            out[torch.tensor(own, device=dev)] = pack
            continue
        buf = torch.empty((len(own), 2, h, w), device=dev, dtype=dt)
        ops.append(dist.P2POp(dist.irecv, buf, src, group))
        recvd.append((own, buf))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    for own, buf in recvd:
        out[torch.tensor(own, device=dev)] = buf
    return out[:, 0:1], out[:, 1:2]


class _HipOps:
    """The product path: fused HIP cost volume slab + HIP soft-argmin."""

    @staticmethod
    def cost_volume_slab(K, R, T, d_min, d_int, feats, batch_size, n_views, d_num, d_scale, d_begin,
                         d_count):
        from .costvolume import warp_and_assemble_cost_volume
        return warp_and_assemble_cost_volume(K, R, T, d_min, d_int, feats, batch_size, n_views,
                                             d_num=d_num, d_scale=d_scale, d_begin=d_begin,
                                             d_count=d_count)

    @staticmethod
    def extract_depth_map(prob, d_batch, n_est):
        from .depthmap import extract_depth_map
        return extract_depth_map(prob, d_batch, n_est)


class DepthShardedMVSNet(nn.Module):
    """Wraps an ``MVSNet``: D-sharded cost volume + owner-targeted exchange + owner-computes
    regulariser.

    ``forward`` returns MVSNet.forward's ``(initial, refined)`` [B, 1, h, w] for the whole batch on
    rank ``dst`` (the owners' maps gathered there, ``gather_depth_maps``) and ``(None, None)`` on the
    other ranks; with ``gather=False`` it returns ``(samples, initial, refined)`` on every rank: the
    samples this rank owns and their maps (``None`` when it owns none).  ``ops`` supplies the slab
    producer and the soft-argmin (default: the HIP kernels).

    ``phase_hook`` (optional callable, name -> None) is called at the END of each phase of a step,
    in order: "encoder", "shard_kernel" (this rank's D-slab of the cost volume), "exchange" (the
    owner-targeted point-to-point exchange), "owner_compute" (regulariser + soft-argmin + refinement
    of the owned samples; nothing on a rank that owns none), "gather" (the depth maps to ``dst``).
    bench.py --mode dshard records a HIP event there, per rank."""

    def __init__(self, net, world, rank, group=None, ops=None, gather=True, dst=0):
        super().__init__()
        self.net = net
        self.world = world
        self.rank = rank
        self.group = group
        self.ops = ops or _HipOps
        self.gather = gather
        self.dst = dst
        self.phase_hook = None

    def _phase(self, name):
        if self.phase_hook is not None:
            self.phase_hook(name)

    def _check_mode(self):
        if torch.is_grad_enabled():
            raise RuntimeError("DepthShardedMVSNet is inference-only: the point-to-point exchange "
                               "carries no gradient (run under torch.no_grad())")
        bns = [m for m in self.net.modules() if isinstance(m, nn.modules.batchnorm._BatchNorm)]
        if any(m.training for m in bns):
            raise RuntimeError("DepthShardedMVSNet needs BatchNorm in eval mode: train-mode batch "
                               "statistics would cover only this rank's samples (model.py:184)")

    def forward(self, nn_input, K_batch, R_batch, T_batch, d_min, d_int, batch_size, n_views):
        self._check_mode()
        c = self.net.cfg
        d_begin, d_count = plane_shard(c.d_num, self.world, self.rank)
        feats = self.net.feature_encoder(nn_input)
        self._phase("encoder")
        slab, d_batch, ref_views = self.ops.cost_volume_slab(
            K_batch, R_batch, T_batch, d_min, d_int, feats, batch_size, n_views, c.d_num, c.d_scale,
            d_begin, d_count)
        self._phase("shard_kernel")
        cv = exchange_to_owners(slab, self.world, self.rank, self.group)
        self._phase("exchange")
        mine = owned_samples(batch_size, self.world, self.rank)
        initial = refined = None
        if mine:
            idx = torch.tensor(mine, device=cv.device)
            prob = self.net.cost_volume_reg(cv)
            d_sel = d_batch.to(cv.device).index_select(0, idx)
            initial = self.ops.extract_depth_map(prob, d_sel, c.n_depth_est)
            dm = d_min.reshape(-1, 1, 1, 1).expand(batch_size, 1, 1, 1).to(cv.device).index_select(0, idx)
            di = d_int.reshape(-1, 1, 1, 1).expand(batch_size, 1, 1, 1).to(cv.device).index_select(0, idx)
            refined = self.net.refine(nn_input, initial, dm, di, ref_views[mine])
        self._phase("owner_compute")
        if not self.gather:
            return mine, initial, refined
        h, w = feats.shape[2:]
        out = gather_depth_maps(initial, refined, batch_size, self.world, self.rank, h, w, self.dst, self.group,
                                feats.device, feats.dtype)
        self._phase("gather")
        return out
