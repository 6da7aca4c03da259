"""Benchmark: depth maps/s of MVSNet.forward on the fused MI355X cost-volume path + warp-kernel HBM GB/s.

Workload (BASELINE.json configs[1]): 3-view DTU geometry, 640x512 images (160x128 features), D=192,
batch 4 per GPU, synthetic N(0,1) images already resident in HBM, real DTU scan-1 cameras
(tests/golden/dtu_scan1_cameras.npz), d_min=425, d_int=1, D_SCALE=25, random-init weights of the
reference architecture (tests/golden/weights.py formula), fp32, BN eval mode, inference (no_grad).

A step = one full MVSNet.forward over one batch (HIP feature encoder -> fused warp+variance HIP
kernel -> 3-D regulariser on its live regions (HIP MFMA region convs) -> HIP softmax
and soft-argmin -> HIP refinement), in exact fp32 arithmetic in every layer (MVSConfig(arithmetic=
"fp32"), the default).  value = depth maps/s over all ranks.

Multi-GPU (torchrun, one process per GPU): --mode samples (default) shards SAMPLES across ranks --
every rank runs its own batch, no collective in the data path, "scaling": "weak".  --mode dshard
runs BASELINE configs[3]: D=256 planes split across ranks, each rank's fused kernel writes its
D-slab, and each sample's slab goes point to point (RCCL send/recv over xGMI,
mvs_amd/depth_shards.py) to the rank that owns the sample, which runs the regulariser.

Also reported (one JSON line, rank 0):
  roofline        the fp32 step's dominant kernel, conv_0_0 (conv3d_k3_narrow_kernel<8>, fp32 VALU with a
                  depth-Winograd transform): its useful convolution flops per launch / its average launch
                  time (HIP events on its stream inside the timed steps) vs the fp32 peak (157.3 TF, the
                  f32 VALU and f32-input MFMA rate); traffic = PMC HBM bytes per launch
                  (profiles/conv0_traffic_<cfg>.json, rocprofv3 --pmc, FETCH_SIZE x2 + WRITE_SIZE)
  warp_kernel     the fused warp + variance kernel (cost_volume_staged_kernel, fp32 channel-quad store)
                  inside the timed steps: algorithmic bytes (features read once + cost volume written
                  once) / launch time vs 8 TB/s -- the metric's "warp-kernel HBM GB/s"; traffic = PMC bytes
  split_f16_step  the opt-in split-fp16 arithmetic (MVSConfig(arithmetic="split_f16"): f16 matrix cores
                  with split operands, narrower than fp32) timed the same way, with its split head's
                  roofline -- never the headline
  cpu_baseline    the oracle (oracle/mvs_oracle.py: the reference's op sequence in torch CPU,
                  per-plane warp loop with torch.cat growth) on ONE sample of the same workload
  hot_path        cost volumes/s of the fused kernel alone
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
# MIOpen find results for the regulariser's convolutions ship with the repo (a text database of
# chosen solvers, tools/miopen_db), so a fresh box skips most of the multi-minute search.  Must be
# set before torch initialises MIOpen.
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(REPO, "tools", "miopen_db"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

for sub in ("deep-multiview-depth-estimation_amd", os.path.join("tests", "golden")):
    sys.path.insert(0, os.path.join(REPO, sub))

from cameras import camera_batch, depth_range  # noqa: E402
from weights import deterministic_state_dict  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec
MFMA_F16_PEAK_TFS = 2500.0   # MI355X_MICROARCH.md: BF16/F16 ~2.5 PF dense
MFMA_F32_PEAK_TFS = 157.3    # f32-input MFMA = f32 vector peak
_T0 = time.perf_counter()


_PHASE = ["start"]


def log(msg):
    """Progress on stderr (stdout carries only the JSON line)."""
    _PHASE[0] = msg
    print("[bench %7.1fs] %s" % (time.perf_counter() - _T0, msg), file=sys.stderr, flush=True)


def _heartbeat():
    # a long phase (first MIOpen call, CPU baseline) still shows progress every 30 s
    while True:
        time.sleep(30.0)
        print("[bench %7.1fs] ... %s" % (time.perf_counter() - _T0, _PHASE[0]), file=sys.stderr,
              flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", choices=("samples", "dshard"), default="samples")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--views", type=int, default=3)
    ap.add_argument("--planes", type=int, default=None)
    ap.add_argument("--height", type=int, default=512)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--kernel-iters", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-planes", type=int, default=None, help="planes for the CPU sample")
    ap.add_argument("--kernel-only", action="store_true", help="skip the end-to-end forward")
    ap.add_argument("--no-extra", action="store_true", help="skip the cfg 3/5 end-to-end fields")
    ap.add_argument("--no-train-step", action="store_true",
                    help="skip the train.py step field (autograd through the full-volume regulariser; "
                         "timed by default at N=1)")
    ap.add_argument("--dist-init", action="store_true",
                    help="create the RCCL process group even at world size 1 (exercises the nccl code path)")
    ap.add_argument("--conv-search", choices=("on", "off"), default="off",
                    help="torch.backends.cudnn.benchmark (MIOpen find) for the regulariser convs")
    return ap.parse_args()


def init_dist(args):
    """One process per GPU: an RCCL ("nccl") process group when WORLD_SIZE > 1, or with --dist-init at
    world size 1 (the RCCL code path of --mode dshard on one GPU), created before any other GPU work."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or args.dist_init:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, torch.device("cuda", local)


def barrier(world):
    if world > 1 or (dist.is_available() and dist.is_initialized()):
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x, world, device):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def timed_steps(step, steps, world, device, hooked=False):
    """``steps`` steps bracketed by a barrier + device synchronisation on both sides: (seconds, {kernel kind:
    average ms}) -- with ``hooked``, HIP events around the step's own kernels (ops.KERNEL_EVENT_HOOK: the
    warp kernel "cost_volume", the fp32 "conv_0_0", the split head "split_head"), recorded on the stream
    each is launched on."""
    from mvs_amd import ops as mvs_ops
    events = []
    stream = torch.cuda.current_stream(device)

    def hook(kind):
        pair = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        for e in pair:   # materialise the HIP event (torch creates it on first record)
            e.record(stream)
        events.append((kind, pair))
        return pair
    with torch.no_grad():
        barrier(world)
        mvs_ops.KERNEL_EVENT_HOOK = hook if hooked else None
        try:
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            barrier(world)
            dt = time.perf_counter() - t0
        finally:
            mvs_ops.KERNEL_EVENT_HOOK = None
    kms = {}
    for kind in sorted(set(k for k, _ in events)):
        ev = [p for k, p in events if k == kind]
        kms[kind] = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
    return dt, kms


DSHARD_PHASES = ("encoder", "shard_kernel", "exchange", "owner_compute", "gather")


def dshard_step(net, world, rank, inputs, B, V, ops=None, group=None):
    """BASELINE configs[3]'s step: mvs_amd.depth_shards.DepthShardedMVSNet around ``net`` (this rank's
    D-slab of the cost volume, the owner-targeted exchange, the owner's regulariser / soft-argmin /
    refinement, the depth maps gathered to rank 0).  Returns (the wrapper, a no-argument step).
    ``ops`` swaps the slab producer / soft-argmin (the CPU gloo test passes the oracle's)."""
    from mvs_amd.depth_shards import DepthShardedMVSNet
    sharded = DepthShardedMVSNet(net, world, rank, group=group, ops=ops)
    return sharded, (lambda: sharded(*inputs, B, V))


def dshard_phase_ms(sharded, step, steps, device, world):
    """This rank's time per phase of the D-sharded step (DSHARD_PHASES, DepthShardedMVSNet.phase_hook),
    averaged over ``steps`` steps: HIP events on the current stream at each phase end on a GPU (a phase
    is the time between its end and the previous one's), wall clock after a synchronising phase end
    on the CPU.  All-gathered: returns [[ms per phase] for every rank] on every rank."""
    cuda = device.type == "cuda"
    sums = [0.0] * len(DSHARD_PHASES)
    for _ in range(steps):
        marks = []

        def mark(name):
            if cuda:
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                marks.append((name, e))
            else:
                marks.append((name, time.perf_counter()))
        mark("start")
        sharded.phase_hook = mark
        try:
            with torch.no_grad():
                step()
        finally:
            sharded.phase_hook = None
        if cuda:
            torch.cuda.synchronize(device)
        names = [n for n, _ in marks]
        assert tuple(names[1:]) == DSHARD_PHASES, names
        for i in range(1, len(marks)):
            a, b = marks[i - 1][1], marks[i][1]
            sums[i - 1] += a.elapsed_time(b) if cuda else 1000.0 * (b - a)
    mine = [v / steps for v in sums]
    if world == 1:
        return [mine]
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    return allr


def make_inputs(B, V, H, W, seed, device):
    h, w = H // 4, W // 4
    K, R, T = camera_batch(B, V, h, w, first_sample=seed)
    d_min, d_int = depth_range(B)
    g = torch.Generator(device="cpu").manual_seed(1000 + seed)
    img = torch.randn(B * V, 3, H, W, generator=g).to(device)
    return img, K.to(device), R.to(device), T.to(device), d_min.to(device), d_int.to(device)


def build_model(D, H, W, device, cv_dtype="float32", arithmetic="fp32"):
    from mvs_amd.config import MVSConfig
    from mvs_amd.model import MVSNet
    net = MVSNet(MVSConfig(d_num=D, in_h=H, in_w=W, cv_dtype=cv_dtype, arithmetic=arithmetic))
    net.load_state_dict(deterministic_state_dict(net.state_dict()))
    return net.to(device).eval()


def time_kernel(B, V, C, h, w, D, device, iters, d_begin=0, d_count=None, bf16=False, quads=False, store="ncdhw"):
    """Fused-kernel timing with HIP events on the launch stream, through the C ABI.

    Returns (main_ms, op_ms, alg_bytes): main_ms = average duration of the main fused kernel
    (events recorded by mvs_cost_volume_fwd_timed right around its launch), op_ms = average
    duration of the whole op (sampling matrices + packing + reference resampling + main kernel).
    store="c4" times the fp32 channel-quad variant (mvs_cost_volume_fwd_c4, what MVSNet.forward's fp32
    inference step runs), "c4_split" the split channel-quad store of the split-fp16 opt-in (same bytes).  bf16=True times the opt-in bf16 cost volume
    (mvs_cost_volume_fwd_bf16): op-level only (main_ms None), algorithmic bytes with a 2-byte
    cost volume."""
    from mvs_amd import _lib, ops
    lib = _lib.load()
    d_count = D if d_count is None else d_count
    K, R, T = camera_batch(B, V, h, w)
    d_min, d_int = depth_range(B)
    K, R, T, d_min, d_int = ops._cams(K, R, T, d_min, d_int, device, B)
    g = torch.Generator(device="cpu").manual_seed(7)
    feat = torch.randn(B * V, C, h, w, generator=g).to(device)
    cv = torch.empty((B, C, d_count, h, w), device=device,
                     dtype=torch.bfloat16 if bf16 else torch.float32)   # (same bytes as the quad layouts)
    ws = torch.empty((lib.mvs_cost_volume_workspace_bytes(B, V, C, h, w, d_count) + 3) // 4,
                     device=device)
    absmax = torch.empty((8,), device=device, dtype=torch.int32)
    stream = torch.cuda.current_stream(device)
    sp = _lib.stream_handle(device)

    def launch(e0=None, e1=None):
        if bf16 and quads:
            st = lib.mvs_cost_volume_fwd_c4_bf16(
                _lib.ptr(feat), _lib.ptr(K), _lib.ptr(R), _lib.ptr(T), _lib.ptr(d_min), _lib.ptr(d_int),
                B, V, C, h, w, d_begin, d_count, 25.0, _lib.ptr(ws), _lib.ptr(cv), sp,
                None if e0 is None else ctypes.c_void_p(e0.cuda_event),
                None if e1 is None else ctypes.c_void_p(e1.cuda_event))
            _lib.check(st, "mvs_cost_volume_fwd_c4_bf16")
            return
        if bf16:
            st = lib.mvs_cost_volume_fwd_bf16(
                _lib.ptr(feat), _lib.ptr(K), _lib.ptr(R), _lib.ptr(T), _lib.ptr(d_min),
                _lib.ptr(d_int), B, V, C, h, w, d_begin, d_count, 25.0, _lib.ptr(ws), _lib.ptr(cv), sp)
            _lib.check(st, "mvs_cost_volume_fwd_bf16")
            return
        evs = (None if e0 is None else ctypes.c_void_p(e0.cuda_event),
               None if e1 is None else ctypes.c_void_p(e1.cuda_event))
        args = (_lib.ptr(feat), _lib.ptr(K), _lib.ptr(R), _lib.ptr(T), _lib.ptr(d_min), _lib.ptr(d_int),
                B, V, C, h, w, d_begin, d_count, 25.0, _lib.ptr(ws), _lib.ptr(cv), sp) + evs
        if store == "c4_split":   # the split cost volume of the split-fp16 opt-in (16-byte elements, bound words)
            st = lib.mvs_cost_volume_fwd_c4_split(*args, _lib.ptr(absmax))
            _lib.check(st, "mvs_cost_volume_fwd_c4_split")
        elif store == "c4":   # the fp32 channel-quad volume the fp32 eval step writes
            st = lib.mvs_cost_volume_fwd_c4(*args)
            _lib.check(st, "mvs_cost_volume_fwd_c4")
        else:
            st = lib.mvs_cost_volume_fwd_timed(*args)
            _lib.check(st, "mvs_cost_volume_fwd_timed")

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(iters)]
    for e0, e1 in ev:   # materialise the HIP events (torch creates them on first record)
        e0.record(stream)
        e1.record(stream)
    op0, op1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    op0.record(stream)
    for e0, e1 in ev:
        launch(e0, e1)
    op1.record(stream)
    torch.cuda.synchronize()
    main_ms = None if (bf16 and not quads) else sum(e0.elapsed_time(e1) for e0, e1 in ev) / iters
    op_ms = op0.elapsed_time(op1) / iters
    alg_bytes = 4.0 * B * V * C * h * w + (2.0 if bf16 else 4.0) * B * C * d_count * h * w
    return main_ms, op_ms, alg_bytes


def time_backward(B, V, C, h, w, D, device, iters=5):
    """The fused op's backward (mvs::cost_volume_backward), called directly after
    one forward, HIP events on the current stream: ms per call in the default mode (fp64 on-chip
    partial sums, fp32 global atomics) and the deterministic mode (64-bit fixed point)."""
    from mvs_amd import ops
    K, R, T = camera_batch(B, V, h, w)
    d_min, d_int = depth_range(B)
    g = torch.Generator(device="cpu").manual_seed(3)
    feat = torch.randn(B * V, C, h, w, generator=g).to(device)
    gcv = torch.randn(B, C, D, h, w, generator=g).to(device)
    _, ws = ops.cost_volume(feat, K, R, T, d_min, d_int, B, V, 0, D, 25.0)
    out = {}
    for det in (False, True):
        ops.cost_volume_backward(feat, ws, gcv, B, V, D, det)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            ops.cost_volume_backward(feat, ws, gcv, B, V, D, det)
        e1.record()
        torch.cuda.synchronize()
        out["deterministic_ms" if det else "bwd_ms"] = e0.elapsed_time(e1) / iters
    # 2 GB of grad_cv read once + features read + gradient written: the HBM floor of the op
    alg = 4.0 * B * C * D * h * w + 8.0 * B * V * C * h * w
    out.update({"alg_bytes": alg, "hbm_floor_ms": alg / (HBM_PEAK_GBS * 1e9) * 1e3,
                "kernel": "cost_volume_bwd_kernel (recompute + LDS footprint accumulation: fp64 "
                          "default / 64-bit fixed point deterministic) + ref_scatter_kernel"})
    del feat, gcv, ws
    return out


KERNEL_CFGS = {   # BASELINE.json configs[2..4]: (B, V, h, w, D, d_count)
    "cfg3": (8, 5, 128, 160, 192, 192),
    "cfg4_shard": (1, 3, 128, 160, 256, 32),
    "cfg5": (1, 3, 296, 400, 256, 256),
}


def kernel_configs(device, iters):
    """Main fused kernel at the other BASELINE configs (live HIP events, as the roofline): the
    channel-quad store of the inference step, NCDHW for the depth shard (the layout the owner
    exchange moves)."""
    out = {}
    for name, (B, V, h, w, D, dc) in KERNEL_CFGS.items():
        quads = dc == D
        k_ms, op_ms, alg = time_kernel(B, V, 32, h, w, D, device, iters, D - dc, dc, store="c4" if quads else "ncdhw")
        gbs = alg / (k_ms * 1e-3) / 1e9
        out[name] = {"B": B, "V": V, "feature_hw": [h, w], "planes": dc, "kernel_ms": k_ms, "op_ms": op_ms,
                     "alg_bytes": alg, "GBps": gbs, "frac": gbs / HBM_PEAK_GBS,
                     "store": "channel-quad" if quads else "NCDHW"}
        torch.cuda.empty_cache()
    return out


E2E_CFGS = {   # BASELINE.json configs[2] and configs[4] end to end: (B, V, D, image H, image W)
    "cfg3": (8, 5, 192, 512, 640),
    "cfg5": (1, 3, 256, 1184, 1600),
}


def e2e_configs(device, steps):
    """MVSNet.forward (BN eval, no_grad, the live-region HIP path of `value`) at cfg 3 (5 views, B=8)
    and cfg 5 (1600x1184 full-resolution images, D=256, B=1): ms/step and depth maps/s on this GPU,
    timed like the headline (warm-up, then `steps` steps between device synchronisations)."""
    out = {}
    for name, (B, V, D, H, W) in E2E_CFGS.items():
        log("e2e %s: B=%d V=%d D=%d %dx%d" % (name, B, V, D, W, H))
        net = build_model(D, H, W, device)
        inputs = make_inputs(B, V, H, W, 0, device)
        with torch.no_grad():
            for _ in range(2):
                net(*inputs, B, V)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                net(*inputs, B, V)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps
        out[name] = {"B": B, "V": V, "planes": D, "image_hw": [H, W], "feature_hw": [H // 4, W // 4],
                     "ms_per_step": 1000.0 * dt, "depth_maps_per_s": B / dt, "steps": steps}
        del net, inputs
        torch.cuda.empty_cache()
    return out


def bf16_step(net32, inputs, B, V, D, H, W, device, world, steps):
    """The reduced-precision opt-in (MVSConfig(cv_dtype="bfloat16")) timed as the
    headline step: the fused kernel stores the cost volume as bf16 channel quads (8 B per 4 channels,
    half the write) and the regulariser's HIP layers read it widened to fp32.  Reported beside the
    fp32 headline with the depth deviation it causes (initial depth vs the fp32 step, same inputs and
    weights); never the headline value."""
    log("bf16 cost-volume opt-in step")
    net = build_model(D, H, W, device, cv_dtype="bfloat16")
    with torch.no_grad():
        ini32 = net32(*inputs, B, V)[0]
        for _ in range(2):
            ini16 = net(*inputs, B, V)[0]
        barrier(world)
        t0 = time.perf_counter()
        for _ in range(steps):
            net(*inputs, B, V)
        barrier(world)
        dt = time.perf_counter() - t0
    rel = ((ini16 - ini32).abs() / ini32.abs()).flatten()
    out = {"ms_per_step": 1000.0 * dt / steps, "value": B * world * steps / dt, "steps": steps,
           "initial_depth_rel_diff_vs_fp32": {"median": rel.median().item(), "p99": rel.quantile(0.99).item()
                                              if rel.numel() <= 16_000_000 else None, "max": rel.max().item(),
                                              "frac_within_1e-4": (rel <= 1e-4).float().mean().item()},
           "note": "cv stored bf16 (RNE of the fp32 variance), fp32 regulariser on the rounded values; "
                   "bit-identical to the fp32 step run on the rounded volume (tests/test_bf16_cost_volume.py)"}
    del net
    torch.cuda.empty_cache()
    return out


def masked_mae_loss(gt, initial, refined):
    """The reference objective (scripts/loss.py:4-41): per sample the mean absolute error of the
    initial and the refined depth over the valid (gt != 0) pixels, summed over both and the batch."""
    mask = (gt != 0).to(gt.dtype)
    valid = mask.sum((1, 2, 3))
    l0 = (mask * (gt - initial).abs()).sum((1, 2, 3)) / valid
    l1 = (mask * (gt - refined).abs()).sum((1, 2, 3)) / valid
    return (l0 + l1).sum()


def train_step_bench(B, V, D, H, W, device, steps):
    """One train.py:86-104 step on the drop-in at the headline workload: model.train(),
    optimizer.zero_grad, MVSNet.forward with autograd (BN batch statistics), the reference loss,
    loss.backward() (HIP cost-volume backward + per-tap rocBLAS GEMMs for the convolutions, tap_gemm.py),
    Adam.step over the
    reference's `model.parameters` list (train.py:160).  Synthetic ground truth: depths uniform over
    the plane range, 10 % invalid (0) pixels."""
    log("train step: B=%d V=%d D=%d %dx%d" % (B, V, D, W, H))
    net = build_model(D, H, W, device).train()
    opt = torch.optim.Adam(net.parameters, lr=1e-3)
    img, K, R, T, d_min, d_int = make_inputs(B, V, H, W, 0, device)
    g = torch.Generator(device="cpu").manual_seed(5)
    gt = 425.0 + 25.0 * D * torch.rand(B, 1, H // 4, W // 4, generator=g)
    gt[torch.rand(B, 1, H // 4, W // 4, generator=g) < 0.1] = 0.0
    gt = gt.to(device)

    def step():
        opt.zero_grad(set_to_none=True)
        ini, ref = net(img, K, R, T, d_min, d_int, B, V)
        loss = masked_mae_loss(gt, ini, ref)
        loss.backward()
        opt.step()
        return loss

    t0 = time.perf_counter()
    step()
    torch.cuda.synchronize()
    first = time.perf_counter() - t0
    n = max(3, steps)   # the first (slow: library initialisation) step is reported on its own
    t0 = time.perf_counter()
    for _ in range(n):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    out = {"B": B, "V": V, "planes": D, "image_hw": [H, W], "ms_per_step": 1000.0 * dt,
           "depth_maps_per_s": B / dt, "steps": n, "first_step_ms": 1000.0 * first,
           "loss": float(loss.item()), "peak_mem_GB": torch.cuda.max_memory_allocated(device) / 1e9,
           "note": "forward (autograd, train-mode BN) + loss.py masked MAE + backward + Adam.step.  Regulariser "
                   "on its live regions under autograd (CostVolumeReg.live_autograd_ok: the same function as the "
                   "full-volume op sequence, float64 gradients equal, tests/test_regulariser_live.py): conv_0_0 "
                   "/ conv_out forward, input and weight gradients on HIP kernels (mvs_amd/narrow_train.py, "
                   "csrc/conv3d_wgrad.hip); the stride-1 and transposed region convolutions' forward and the "
                   "encoder convs' forward on the HIP kernels (mvs_amd/region_train.py, tap_gemm.conv2d_hip_fwd), "
                   "their backward and the stride-2 convs as per-tap rocBLAS GEMMs on dense boxes "
                   "(mvs_amd/tap_gemm.py; the three stride-2 convs as one); cost volume backward on "
                   "mvs::cost_volume_backward"}
    del net, opt
    torch.cuda.empty_cache()
    return out


def head_work(B, V, D, h, w, kind="split_head"):
    """Work of one head launch at the eval step's regions: executed f16 MFMA flops, the fp32
    convolution flops they compute (conv_0_0 + conv_1_0, model.py:101,103), and the algorithmic HBM
    bytes.  kind "split_head" (the default path, ops.split_head): the split cost volume read once
    (128 B per voxel: 8 channel quads x hi/lo fp16), y0 and the conv_1_0 window region written once.
    kind "cv_head" (opt-in fused head): pixel-major padded features + resampled reference views read
    once; y0, the window region and the split volume on conv_2_0's input box written once."""
    from mvs_amd import model as M
    from mvs_amd.config import pad_outpad
    n = (D, h, w)
    pad = pad_outpad(D, h, w)[0]
    full = tuple((0, d - 1) for d in n)
    b_reg = M._tconv_input_region(full, n, pad)
    c2 = M._tconv_input_region(b_reg, n, pad)
    h1, h2 = M._grow(b_reg, n, 1), M._grow(c2, n, 1)
    lo = [max(2 * a - p, 0) for (a, _), p in zip(h2, pad)]
    hi = [min(2 * b - p + 2, d - 1) + 1 for (_, b), p, d in zip(h2, pad, n)]
    vox = D * h * w
    win = int(np.prod([b - a + 1 for a, b in h1]))
    box = int(np.prod([b - a for a, b in zip(lo, hi)]))
    out_bytes = B * (vox * 8 * 4 + win * 16 * 4)
    if kind == "split_head":
        hbm = B * vox * 128 + out_bytes
    else:
        hbm = B * V * (h + 2) * (w + 2) * 128 + B * h * w * 128 + out_bytes + B * box * 8 * 16
    return {"mfma_flops": B * (vox * 55296 + win * 82944),
            "alg_flops": B * (vox * 8 * 32 * 27 * 2 + win * 16 * 32 * 27 * 2),
            "hbm_bytes": hbm,
            "regions": {"conv_1_0_windows": list(h1), "scv_box": [lo, hi]}}


def conv0_flops(B, D, h, w):
    """Useful fp32 flops of conv_0_0 (model.py:101: Conv3d(32, 8, 3, padding 1) over the whole volume)."""
    return float(B) * D * h * w * 8 * 32 * 27 * 2


def time_conv0_isolated(B, D, h, w, device, iters=10):
    """conv_0_0's kernel alone (the fp32 eval step's roofline kernel: conv3d_k3, channel-quad input, depth
    Winograd, BN_0 + ReLU), back-to-back launches on one stream, HIP events: ms per launch -- beside its
    in-step duration, which the concurrent region chain stretches (they share the CUs)."""
    from mvs_amd.ops import conv3d_k3
    g = torch.Generator(device="cpu").manual_seed(11)
    cv4 = torch.rand((B, 8, D, h, w, 4), generator=g).to(device)
    wt = (torch.randn(8, 32, 3, 3, 3, generator=g) * 0.05).to(device)
    bn = [torch.ones(8, device=device), torch.zeros(8, device=device), torch.zeros(8, device=device)]
    with torch.no_grad():
        for _ in range(2):
            conv3d_k3(cv4, wt, *bn, in_c4=True, wino_z=True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            conv3d_k3(cv4, wt, *bn, in_c4=True, wino_z=True)
        e1.record()
        torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    del cv4
    torch.cuda.empty_cache()
    return ms


def conv0_traffic(tag, kind="conv0"):
    """PMC HBM bytes per fp32 conv_0_0 (kind "conv0") or fused fp32 head ("conv_head_fp32") launch
    (profiles/<kind>_traffic_<tag>.json, rocprofv3 --pmc), or None."""
    path = os.path.join(REPO, "profiles", "%s_traffic_%s.json" % (kind, tag))
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get("hbm_bytes_per_launch")


def head_traffic(tag, kind="split_head"):
    """PMC HBM bytes per head launch (profiles/, rocprofv3 --pmc), or None."""
    path = os.path.join(REPO, "profiles", "%s_traffic_%s.json" % ("head" if kind == "cv_head" else kind, tag))
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get("hbm_bytes_per_launch")


def load_traffic(tag):
    p = os.path.join(REPO, "profiles", "traffic_%s.json" % tag)
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    return None


def host_cpus():
    """CPUs this process may use: its affinity set, capped by a cgroup-v2 CPU quota (a GPU box
    shows the whole machine in os.cpu_count() but grants one GPU's share), plus lscpu facts."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    info = {"os_cpu_count": os.cpu_count(), "affinity": n, "cgroup_quota": quota}
    try:
        import subprocess
        txt = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in txt.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core"):
                info[k.strip()] = v.strip()
    except (OSError, ValueError):
        pass
    return min(n, quota) if quota else n, info


def _median(fn, reps=3, warmup=True):
    import statistics
    if warmup:
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def cpu_baseline(V, H, W, D):
    """The oracle (oracle/mvs_oracle.py: the reference's op sequence in torch CPU, per-plane warp
    loop with torch.cat growth; within 6 % of the imported reference at config 1 in the survey
    container, profiles/cpu_calibration_r02.json) on the host cores available to this job,
    BASELINE.md's CPU-baseline plan on bounded samples:
      value  cfg 2 (D=192, 640x512, V=3) full MVSNet.forward of ONE sample, median of 3 (the
             config-1 runs before it warm every op up);
      legs   config 1 (D=48) full forward, one warm-up + median of 3; cfg 2 warp + variance only
             (homography_warping + assemble_cost_volume), one sample, median of 3.
    cfg 5 is skipped (the reference's O(D^2) torch.cat makes it ~1.5 TB of copies per sample)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import mvs_oracle
    threads, info = host_cpus()
    torch.set_num_threads(threads)
    from mvs_amd.config import MVSConfig
    from mvs_amd.model import MVSNet
    out = {}
    with torch.no_grad():
        for tag, d in (("cfg1", 48), ("cfg2", D)):
            net = MVSNet(MVSConfig(d_num=d, in_h=H, in_w=W), device=torch.device("cpu"))
            net.load_state_dict(deterministic_state_dict(net.state_dict()))
            net.eval()
            img, K, R, T, d_min, d_int = make_inputs(1, V, H, W, 0, torch.device("cpu"))
            log("cpu baseline: %s full forward (D=%d, %d threads)" % (tag, d, threads))
            out[tag + "_forward_s"] = _median(lambda: mvs_oracle.mvsnet_forward(
                net, img, K, R, T, d_min, d_int, 1, V, d, (H // 4, W // 4), concat_growth=True),
                warmup=(tag == "cfg1"))
            if tag == "cfg2":
                feats = net.feature_encoder(img)
                log("cpu baseline: cfg2 warp + variance")
                out["cfg2_warp_variance_s"] = _median(lambda: mvs_oracle.assemble_cost_volume(
                    mvs_oracle.homography_warping(K, R, T, d_min, d_int, feats, 1, V, d,
                                                  concat_growth=True)[0], V), warmup=False)
    dt = out["cfg2_forward_s"]
    return {"value": 1.0 / dt, "unit": "depth maps/s", "cores": threads, "kind": "port",
            "sample": "1 sample (B=1, V=%d, %dx%d, D=%d) of the workload, full MVSNet.forward on the "
                      "oracle (reference op sequence incl. per-plane warp loop with torch.cat growth), "
                      "median of 3, torch %s CPU, %d threads: %.1f s" % (V, W, H, D, torch.__version__,
                                                                        threads, dt),
            "legs": {"cfg1_forward_s": out["cfg1_forward_s"],
                     "cfg1_depth_maps_per_s": 1.0 / out["cfg1_forward_s"],
                     "cfg2_forward_s": dt,
                     "cfg2_warp_variance_s": out["cfg2_warp_variance_s"],
                     "cfg2_warp_variance_cost_volumes_per_s": 1.0 / out["cfg2_warp_variance_s"]},
            "host": info, "calibration": "profiles/cpu_calibration_r02.json"}


def main():
    threading.Thread(target=_heartbeat, daemon=True).start()
    args = parse()
    world, rank, device = init_dist(args)
    V, H, W = args.views, args.height, args.width
    h, w, C = H // 4, W // 4, 32
    if args.mode == "samples":
        B = args.batch or 4
        D = args.planes or 192
    else:
        B = args.batch or 1
        D = args.planes or 256
        if D % world:
            raise SystemExit("D=%d not divisible by world size %d" % (D, world))
    torch.backends.cudnn.benchmark = args.conv_search == "on"

    result = {}
    ms_step = None
    if not args.kernel_only:
        log("building model (D=%d, %dx%d)" % (D, H, W))
        net = build_model(D, H, W, device)
        # samples mode: every rank its own batch; dshard: ONE batch, replicated on every rank
        inputs = make_inputs(B, V, H, W, rank if args.mode == "samples" else 0, device)
        if args.mode == "samples":
            step = lambda: net(*inputs, B, V)
        else:
            sharded, step = dshard_step(net, world, rank, inputs, B, V)
        # the main fused kernel's launches inside the timed steps, bracketed by HIP events on its
        # launch stream (ops.KERNEL_EVENT_HOOK -> mvs_cost_volume_fwd_c4's event arguments)
        with torch.no_grad():
            for i in range(args.warmup):
                step()
                torch.cuda.synchronize()
                log("warmup step %d/%d done" % (i + 1, args.warmup))
        dt, result["step_kernel_ms"] = timed_steps(step, args.steps, world, device,
                                                   hooked=args.mode == "samples")
        log("timed %d steps: %.2f ms/step" % (args.steps, 1000.0 * dt / args.steps))
        if args.mode == "dshard":
            # the same step phase by phase, per rank (not part of the timed region above)
            result["dshard_phases"] = dshard_phase_ms(sharded, step, max(1, min(args.steps, 5)), device, world)
            log("dshard phases (ms, this rank): %s" % dict(zip(DSHARD_PHASES, result["dshard_phases"][rank])))
        dt = max_over_ranks(dt, world, device)
        ms_step = 1000.0 * dt / args.steps
        maps_per_step = B * world if args.mode == "samples" else B
        result["value"] = maps_per_step * args.steps / dt
        if args.mode == "samples":
            # the opt-in split-fp16 arithmetic (MVSConfig(arithmetic="split_f16"): the f16 matrix cores with
            # split operands, the split cost volume, the split head; narrower than fp32)
            # timed the same way: reported beside value, never as value
            net.set_arithmetic("split_f16")
            with torch.no_grad():
                for _ in range(2):
                    step()
                torch.cuda.synchronize()
            dts, kms = timed_steps(step, args.steps, world, device, hooked=True)
            net.set_arithmetic("fp32")
            dts = max_over_ranks(dts, world, device)
            result["split_f16"] = {"ms_per_step": 1000.0 * dts / args.steps,
                                   "value": maps_per_step * args.steps / dts, "step_kernel_ms": kms}
            log("split-fp16 opt-in step: %.2f ms/step" % result["split_f16"]["ms_per_step"])
        # the same step with the regulariser over the WHOLE volume (CostVolumeReg.forward_full,
        # the reference's op sequence) instead of its eval-mode live regions: reported beside
        # value so the gain of the live-region evaluation is visible
        net.cost_volume_reg.live_region = False
        full_steps = max(1, min(args.steps, 5))
        with torch.no_grad():
            step()
            barrier(world)
            t0 = time.perf_counter()
            for _ in range(full_steps):
                step()
            barrier(world)
            dtf = time.perf_counter() - t0
        dtf = max_over_ranks(dtf, world, device)
        result["full"] = {"ms_per_step": 1000.0 * dtf / full_steps, "value": maps_per_step * full_steps / dtf,
                          "steps": full_steps}
        log("full-volume regulariser: %.2f ms/step" % result["full"]["ms_per_step"])
        net.cost_volume_reg.live_region = True
        # test.py:53,61: the reference's test driver runs the model in TRAIN mode under no_grad
        # (BatchNorm normalises with batch statistics over the whole volume, so the eval-mode
        # live-region shortcut does not apply): timed as its own field, fp32 and split-fp16
        if args.mode == "samples":
            net.train()
            train_steps = max(1, min(args.steps, 10))   # 10 steps keep the figure stable
            for arith in ("fp32", "split_f16"):
                net.set_arithmetic(arith)
                with torch.no_grad():
                    for _ in range(2):
                        step()
                    barrier(world)
                    t0 = time.perf_counter()
                    for _ in range(train_steps):
                        step()
                    barrier(world)
                    dtt = time.perf_counter() - t0
                dtt = max_over_ranks(dtt, world, device)
                result["train_bn" if arith == "fp32" else "train_bn_split_f16"] = {
                    "ms_per_step": 1000.0 * dtt / train_steps, "value": B * world * train_steps / dtt,
                    "steps": train_steps}
                log("train-mode BN step (test.py:61), %s: %.2f ms/step" % (arith, 1000.0 * dtt / train_steps))
            net.set_arithmetic("fp32")
            if not args.no_extra:
                net.eval()
                result["bf16"] = bf16_step(net, inputs, B, V, D, H, W, device, world, args.steps)
        del net

    # fused kernel timing (this rank's share of planes in dshard mode)
    d_count = D if args.mode == "samples" else D // world
    log("timing the fused kernel")
    # samples mode: the fp32 channel-quad store the eval step feeds the regulariser with; dshard mode:
    # the NCDHW slabs the owner exchange moves
    store = "c4" if args.mode == "samples" else "ncdhw"
    k_ms, op_ms, alg = time_kernel(B, V, C, h, w, D, device, args.kernel_iters, 0, d_count, store=store)
    k_ms = max_over_ranks(k_ms, world, device)
    op_ms = max_over_ranks(op_ms, world, device)
    nc_ms, nc_op_ms, _ = time_kernel(B, V, C, h, w, D, device, args.kernel_iters, 0, d_count)
    nc_ms = max_over_ranks(nc_ms, world, device)
    # warp-kernel duration: its launches inside the timed steps
    step_k = result.get("step_kernel_ms", {})
    iso_ms = k_ms
    if "cost_volume" in step_k:
        k_ms = max_over_ranks(step_k["cost_volume"], world, device)
    gbs = alg / (k_ms * 1e-3) / 1e9
    tag = "b%dv%dd%dh%dw%d" % (B, V, d_count, h, w)
    traffic = load_traffic(tag)
    conv0_ms = max_over_ranks(step_k["conv_0_0"], world, device) if "conv_0_0" in step_k else None
    conv0_iso_ms = max_over_ranks(time_conv0_isolated(B, D, h, w, device), world, device) if conv0_ms else None
    head32_ms = max_over_ranks(step_k["conv_head"], world, device) if "conv_head" in step_k else None
    split = result.get("split_f16")
    head_ms = split["step_kernel_ms"].get("split_head") if split else None
    if head_ms is not None:
        head_ms = max_over_ranks(head_ms, world, device)

    if rank != 0:
        if dist.is_initialized():
            dist.destroy_process_group()
        return
    out = {
        "metric": "depth maps/sec + warp-kernel HBM GB/s, 3-view 640x512 D=192, 1/2/4/8 GPU",
        "value": result.get("value"),
        "unit": "depth maps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak" if args.mode == "samples" else "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic N(0,1) images resident in HBM, real DTU scan-1 cameras, random-init "
                "weights; BN eval mode, live-region regulariser (train-mode BN as in test.py:61: "
                "field train_bn)",
        "config": {"workload": "cfg%d: %d-view %dx%d D=%d batch=%d per %s, BN eval, live-region "
                               "regulariser, fp32 arithmetic" % (
                       2 if args.mode == "samples" else 4, V, W, H, D, B,
                       "GPU" if args.mode == "samples" else "job (D sharded)"),
                   "global_batch": B * (world if args.mode == "samples" else 1),
                   "views": V, "planes": D, "image_hw": [H, W], "feature_hw": [h, w],
                   "parallelism": ("samples%d" % world) if args.mode == "samples" else ("dshard%d" % world)},
        "arithmetic": ("exact fp32 in every layer of the timed step (MVSConfig(arithmetic='fp32'), the default): "
                       "fp32 cost volume (the reference's torch-CPU law, bit for bit given the sampling matrices), "
                       "2-D convolutions on fp32 VALU kernels, conv_0_0 / conv_out on fp32 VALU kernels (conv_0_0 "
                       "with a depth-Winograd F(2,3) transform), every region convolution on the f32-input matrix "
                       "cores (v_mfma_f32_16x16x4_f32: each product and sum rounded as an fmaf chain), fp32 "
                       "softmax / soft-argmin / refinement"),
        "warp_kernel": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": gbs / HBM_PEAK_GBS,
                        "traffic": None if traffic is None else traffic.get("hbm_bytes_per_launch"),
                        "kernel": "cost_volume_staged_kernel<V=%d, planes=8, %s>" % (
                            V, "fp32 channel-quad store (16 B per voxel and 4 channels)" if store == "c4"
                            else "NCDHW store"), "kernel_ms": k_ms,
                        "alg_bytes_per_launch": alg,
                        "timing": ("HIP events around each launch inside the %d timed steps" % args.steps
                                   if "cost_volume" in step_k else "HIP events, isolated launches"),
                        "isolated_kernel_ms": iso_ms,
                        "ncdhw_store": {"kernel_ms": nc_ms, "op_ms": nc_op_ms,
                                        "frac": alg / (nc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}},
        "hot_path": {"cost_volumes_per_s": B / (op_ms * 1e-3), "op_ms": op_ms,
                     "op": "mvs_cost_volume_fwd%s: prologue kernel (sampling matrices + channel-quad "
                           "packing + reference resampling) + cost_volume_staged kernel" % (
                               "_c4" if store == "c4" else ""),
                     "op_GBps": alg / (op_ms * 1e-3) / 1e9},
    }
    if head32_ms is not None:
        # the fp32 step's dominant kernel: conv_0_0 (model.py:101, whole volume) + BN_0 + ReLU on the fp32 VALU
        # and conv_1_0 (model.py:103, 32 -> 16 stride 2 on its live region) + BN_1 + ReLU on the f32-input
        # matrix cores in ONE kernel over the fp32 channel-quad volume (ops.conv_head_fp32)
        hw_ = head_work(B, V, D, h, w, "split_head")
        fl = hw_["alg_flops"]
        tf = fl / (head32_ms * 1e-3) / 1e12
        out["roofline"] = {
            "bound": "mfma", "achieved": tf, "peak": MFMA_F32_PEAK_TFS, "unit": "TFLOP/s", "frac": tf / MFMA_F32_PEAK_TFS,
            "traffic": conv0_traffic(tag, "conv_head_fp32"),
            "kernel": "conv3d_k3_narrow_kernel<8, wino_z, C1> (conv_0_0 fp32 VALU + conv_1_0 fp32 MFMA)",
            "kernel_ms": head32_ms, "flops_per_launch": fl,
            "timing": "HIP events around each launch inside the %d timed steps (on its side stream, concurrent "
                      "with the region convolutions)" % args.steps,
            "flops": "useful fp32 convolution flops: conv_0_0 B*D*h*w x 8 x 32 x 27 x 2 + conv_1_0 (its live-region "
                     "windows) x 16 x 32 x 27 x 2 (the direct convolutions'; the depth-Winograd conv_0_0 executes 2/3 "
                     "of its multiplies) against the fp32 compute peak: 157.3 TF is both the f32 VALU rate and the "
                     "f32-input MFMA rate (MI355X_MICROARCH.md), so 'mfma' names the fp32 compute roof (the two "
                     "pipes co-issue, so the kernel's own ceiling is above it)",
            "regions": hw_["regions"],
            "hbm": {"alg_bytes_per_launch": 4.0 * B * D * h * w * (32 + 8),
                    "GBps": 4.0 * B * D * h * w * 40 / (head32_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                    "note": "the fp32 cost volume in once, y0 out once (y1 is 1/16 of y0's bytes)"}}
    elif conv0_ms is not None:
        # the fp32 step's dominant kernel: conv_0_0 (model.py:101, 32 -> 8 over the whole volume + BN_0 +
        # ReLU) on the fp32 VALU kernel, concurrent with the region convolutions on the fp32 matrix cores
        fl = conv0_flops(B, D, h, w)
        tf = fl / (conv0_ms * 1e-3) / 1e12
        out["roofline"] = {
            "bound": "mfma", "achieved": tf, "peak": MFMA_F32_PEAK_TFS, "unit": "TFLOP/s", "frac": tf / MFMA_F32_PEAK_TFS,
            "traffic": conv0_traffic(tag), "kernel": "conv3d_k3_narrow_kernel<8, wino_z> (conv_0_0, fp32 VALU)",
            "kernel_ms": conv0_ms, "flops_per_launch": fl,
            "timing": "HIP events around each launch inside the %d timed steps (on its side stream, concurrent "
                      "with the region convolutions)" % args.steps,
            "flops": "useful fp32 convolution flops B*D*h*w x 8 x 32 x 27 x 2 (the direct convolution's; the "
                     "depth-Winograd kernel executes 2/3 of the multiplies) against the fp32 compute peak: 157.3 "
                     "TF is both the f32 VALU rate and the f32-input MFMA rate (MI355X_MICROARCH.md), so 'mfma' "
                     "names the fp32 compute roof",
            "hbm": {"alg_bytes_per_launch": 4.0 * B * D * h * w * (32 + 8),
                    "GBps": 4.0 * B * D * h * w * 40 / (conv0_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                    "note": "the fp32 cost volume in once, y0 out once"},
            "isolated_kernel_ms": conv0_iso_ms,
            "isolated_frac": fl / (conv0_iso_ms * 1e-3) / 1e12 / MFMA_F32_PEAK_TFS,
            "isolated_note": "the same kernel alone (back-to-back launches, bench.time_conv0_isolated): in the step it "
                             "runs beside the region convolutions on a side stream and shares the CUs with them"}
    else:
        out["roofline"] = dict(out["warp_kernel"])
    if split is not None:
        # the opt-in split-fp16 arithmetic: never the headline (narrower than fp32)
        sp = {"ms_per_step": split["ms_per_step"], "value": split["value"], "unit": "depth maps/s",
              "dtype": "f16x2-split (fp16 hi + lo parts of power-of-two-scaled fp32 operands on the f16 matrix "
                       "cores, fp32 accumulation; narrower than fp32)",
              "note": "MVSConfig(arithmetic='split_f16'), opt-in: encoder / refinement / regulariser convolutions "
                      "on v_mfma_f32_16x16x32_f16 with split operands (22 significant bits per operand, 3-4 partial "
                      "products), the cost volume stored as its fp16 parts and read once by the split head; element "
                      "contract |x - (hi + lo) 2^-e| <= 2^-22 |x| + 2^-37 B^2 (an absolute floor below ~1e-5 of a "
                      "tensor's bound: tests/test_split_conv.py::test_split_conv_dynamic_range, DESIGN.md 3.5)",
              "step_kernel_ms": split["step_kernel_ms"]}
        if head_ms is not None:
            hw_ = head_work(B, V, D, h, w, "split_head")
            alg_tf = hw_["alg_flops"] / (head_ms * 1e-3) / 1e12
            exe_tf = hw_["mfma_flops"] / (head_ms * 1e-3) / 1e12
            sp["roofline"] = {
                "bound": "mfma", "achieved": exe_tf, "peak": MFMA_F16_PEAK_TFS, "unit": "TFLOP/s",
                "frac": exe_tf / MFMA_F16_PEAK_TFS, "traffic": head_traffic(tag, "split_head"),
                "kernel": "cv_head_kernel<2, PRESPLIT>", "kernel_ms": head_ms,
                "timing": "HIP events around each launch inside the %d timed split-fp16 steps" % args.steps,
                "flops_per_launch": hw_["mfma_flops"],
                "flops": "executed f16 matrix-core flops: conv_0_0 2 v_mfma_f32_16x16x32_f16 per (16 voxels, tap), "
                         "conv_1_0 3 per (16 windows, tap)",
                "useful_fp32_conv_flops": {"flops_per_launch": hw_["alg_flops"], "tflops": alg_tf},
                "hbm": {"alg_bytes_per_launch": hw_["hbm_bytes"], "GBps": hw_["hbm_bytes"] / (head_ms * 1e-3) / 1e9,
                        "peak": HBM_PEAK_GBS, "frac": hw_["hbm_bytes"] / (head_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                        "note": "the split cost volume in (once); y0 and y1 out"},
                "regions": hw_["regions"]}
        out["split_f16_step"] = sp
    if "dshard_phases" in result:
        out["dshard_phases"] = {
            "phases": list(DSHARD_PHASES), "ms_per_rank": result["dshard_phases"],
            "note": "per rank, mean over up to 5 extra steps after the timed ones (HIP events on the current "
                    "stream at each phase end): encoder, this rank's D-slab kernel (shard_kernel), the "
                    "owner-targeted point-to-point exchange (exchange, incl. waiting for the slowest sender), "
                    "the owner's regulariser + soft-argmin + refinement (owner_compute; 0 on ranks owning no "
                    "sample), the depth maps to rank 0 (gather)"}
    if "full" in result:
        out["full_volume_regulariser"] = dict(result["full"], unit="depth maps/s", note=(
            "same step with CostVolumeReg.forward_full (every voxel of every level, as "
            "model.py:100-126 computes it: MIOpen, HIP conv_0_0/conv_out); value uses forward_live "
            "(eval BN: only the regions whose values reach the output; same sums, fp32 summation "
            "order may differ)"))
    if "train_bn" in result:
        out["train_bn"] = dict(result["train_bn"], unit="depth maps/s", dtype="f32", note=(
            "test.py:53,61 mode: model.train() under no_grad, BatchNorm batch statistics over the "
            "whole volume and running-statistic updates, exact on live regions "
            "(CostVolumeReg.forward_live_train, DESIGN.md 5b); fp32 arithmetic"))
    if "train_bn_split_f16" in result:
        out["train_bn_split_f16"] = dict(result["train_bn_split_f16"], unit="depth maps/s", dtype="f16x2-split",
                                         note="train_bn with MVSConfig(arithmetic='split_f16') (opt-in)")
    # backward of the fused op (train.py:103): informational
    log("timing the backward")
    out["cost_volume_backward"] = time_backward(B, V, C, h, w, d_count, device)
    if args.mode == "samples":
        log("timing the fused kernel at cfg 3/4/5")
        out["kernel_configs"] = kernel_configs(device, max(5, args.kernel_iters // 2))
        if not args.kernel_only and not args.no_extra:
            out["e2e_configs"] = e2e_configs(device, max(3, min(args.steps, 10)))
        if not args.no_train_step and world == 1:
            log("timing the train.py step")
            out["train_step"] = train_step_bench(B, V, D, H, W, device, 3)
    # opt-in bf16 cost volume: informational, not the headline (reduced precision)
    _, bf_op_ms, bf_alg = time_kernel(B, V, C, h, w, D, device, args.kernel_iters, 0, d_count, bf16=True)
    q_ms, q_op_ms, q_alg = time_kernel(B, V, C, h, w, D, device, args.kernel_iters, 0, d_count, bf16=True,
                                       quads=True)
    out["bf16_cv_opt_in"] = {"ncdhw_op_ms": bf_op_ms, "alg_bytes_per_launch": bf_alg,
                             "ncdhw_op_GBps": bf_alg / (bf_op_ms * 1e-3) / 1e9,
                             "channel_quad_kernel_ms": q_ms, "channel_quad_op_ms": q_op_ms,
                             "channel_quad_GBps": q_alg / (q_ms * 1e-3) / 1e9,
                             "cost_volumes_per_s": B / (q_op_ms * 1e-3)}
    if "bf16" in result:
        out["bf16_cv_opt_in"]["step"] = result["bf16"]
    if not args.no_cpu_baseline and world == 1:
        log("cpu baseline (oracle, one sample)")
        out["cpu_baseline"] = cpu_baseline(V, H, W, args.cpu_planes or D)
    else:
        out["cpu_baseline"] = None
    print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
