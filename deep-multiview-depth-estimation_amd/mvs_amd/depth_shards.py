"""Depth-plane sharding of the cost volume across the GPUs of one node (BASELINE configs[3]).

The fused warp+variance is independent per (sample, plane, pixel), so rank r of P computes planes
[r*D/P, (r+1)*D/P) with no communication (the kernel's ``d_begin``/``d_count``), from replicated
features and cameras.  The 3-D regulariser is NOT D-local (stride-2 convs with padding D/2+1 remap
planes non-locally, softmax and the soft-argmin span all D; SURVEY.md §8 e), so the parity-preserving
exchange is an all-gather of the cost-volume D-slabs (RCCL over xGMI when the process group is
``nccl``), after which the rank that owns a sample (b mod P) runs the regulariser and soft-argmin.

Reference: there is no multi-GPU path in the reference (single device, ``config.py:24``); this
module reproduces ``model.py:168-207`` exactly for every owned sample (BN eval mode).
"""
import torch
import torch.distributed as dist
import torch.nn as nn

from .costvolume import warp_and_assemble_cost_volume
from .depthmap import extract_depth_map


def plane_shard(d_num, world, rank):
    """[begin, count) of the planes rank ``rank`` computes; D must split evenly."""
    if d_num % world:
        raise ValueError("d_num=%d does not split over %d ranks" % (d_num, world))
    count = d_num // world
    return rank * count, count


def owned_samples(batch_size, world, rank):
    """Samples whose regulariser/soft-argmin this rank runs (round-robin)."""
    return [b for b in range(batch_size) if b % world == rank]


def gather_depth_slabs(slab, world, group=None):
    """All-gather [B, C, Dl, h, w] slabs (rank order = plane order) into [B, C, world*Dl, h, w]."""
    if world == 1:
        return slab
    slab = slab.contiguous()
    backend = dist.get_backend(group)
    if backend == "nccl":
        buf = torch.empty((world,) + tuple(slab.shape), dtype=slab.dtype, device=slab.device)
        dist.all_gather_into_tensor(buf, slab, group=group)
    else:
        parts = [torch.empty_like(slab) for _ in range(world)]
        dist.all_gather(parts, slab, group=group)
        buf = torch.stack(parts)
    b, c, dl, h, w = slab.shape
    return buf.permute(1, 2, 0, 3, 4, 5).reshape(b, c, world * dl, h, w)


class DepthShardedMVSNet(nn.Module):
    """Wraps an ``MVSNet``: sharded cost volume + all-gather + owner-computes regulariser.

    ``forward`` returns ``(samples, initial, refined)``: the indices of the samples this rank owns
    and their depth maps ([len(samples), 1, h, w] each; empty when the rank owns none)."""

    def __init__(self, net, world, rank, group=None):
        super().__init__()
        self.net = net
        self.world = world
        self.rank = rank
        self.group = group

    def forward(self, nn_input, K_batch, R_batch, T_batch, d_min, d_int, batch_size, n_views):
        c = self.net.cfg
        d_begin, d_count = plane_shard(c.d_num, self.world, self.rank)
        feats = self.net.feature_encoder(nn_input)
        slab, d_batch, ref_views = warp_and_assemble_cost_volume(
            K_batch, R_batch, T_batch, d_min, d_int, feats, batch_size, n_views,
            d_num=c.d_num, d_scale=c.d_scale, d_begin=d_begin, d_count=d_count)
        cv = gather_depth_slabs(slab, self.world, self.group)
        mine = owned_samples(batch_size, self.world, self.rank)
        if not mine:
            return mine, None, None
        idx = torch.tensor(mine, device=cv.device)
        prob = self.net.cost_volume_reg(cv.index_select(0, idx))
        d_sel = d_batch.index_select(0, idx)
        initial = extract_depth_map(prob, d_sel, c.n_depth_est)
        dm = d_min.reshape(-1, 1, 1, 1).expand(batch_size, 1, 1, 1).to(cv.device).index_select(0, idx)
        di = d_int.reshape(-1, 1, 1, 1).expand(batch_size, 1, 1, 1).to(cv.device).index_select(0, idx)
        refined = self.net.refine(nn_input, initial, dm, di, ref_views[mine])
        return mine, initial, refined
