"""Populate MIOpen's user find-db for every convolution MIOpen still runs: the full-volume regulariser
(CostVolumeReg.forward_full, the reference op sequence the parity tests compare against) at the
BASELINE workloads, and the forward + backward of the train.py step (autograd runs the modules).
Each shape is found once with torch.backends.cudnn.benchmark = True (exhaustive MIOpen find); the db
files are left in $MIOPEN_USER_DB_PATH for tools/miopen_db, so a fresh box (tests, bench) skips the
search -- and immediate mode never falls back to MIOpen's naive kernels, which run these 3-D shapes
for minutes.

Usage (GPU box): MIOPEN_USER_DB_PATH=gpurun_out/miopen_db python tools/miopen_find.py [names...]
"""
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402

# name -> (B, V, D, H, W, what)
SHAPES = {
    "cfg2_full": (4, 3, 192, 512, 640, "full"),
    "cfg3_full": (8, 5, 192, 512, 640, "full"),
    "cfg5_full": (1, 3, 256, 1184, 1600, "full"),
    "cfg1_full": (1, 3, 48, 512, 640, "full"),
    "cfg1_train": (1, 3, 48, 512, 640, "train"),
    "smooth_train": (2, 3, 16, 256, 320, "train"),
    "cfg2_train": (4, 3, 192, 512, 640, "train"),
    "cfg5_live_torch": (1, 3, 256, 1184, 1600, "live_torch"),
}


def heartbeat():
    t0 = time.time()
    while True:
        time.sleep(20)
        print("... find running %.0f s" % (time.time() - t0), flush=True)


def run(name, dev):
    B, V, D, H, W, what = SHAPES[name]
    net = bench.build_model(D, H, W, dev)
    img, K, R, T, d_min, d_int = bench.make_inputs(B, V, H, W, 0, dev)
    t = time.time()
    if what in ("full", "live_torch"):
        from mvs_amd import warp_and_assemble_cost_volume
        with torch.no_grad():
            feats = net.feature_encoder(img)
            cv, _, _ = warp_and_assemble_cost_volume(K, R, T, d_min, d_int, feats, B, V, d_num=D)
            reg = net.cost_volume_reg
            for _ in range(2):
                reg.forward_full(cv) if what == "full" else reg.forward_live_torch(cv)
    else:
        net.train()
        opt = torch.optim.Adam(net.parameters, lr=1e-3)
        gt = torch.full((B, 1, H // 4, W // 4), 600.0, device=dev)
        for _ in range(2):
            opt.zero_grad(set_to_none=True)
            ini, ref = net(img, K, R, T, d_min, d_int, B, V)
            bench.masked_mae_loss(gt, ini, ref).backward()
            opt.step()
    torch.cuda.synchronize()
    print("%s: %.1f s" % (name, time.time() - t), flush=True)
    del net
    torch.cuda.empty_cache()


def main():
    threading.Thread(target=heartbeat, daemon=True).start()
    print("db", os.environ.get("MIOPEN_USER_DB_PATH"), flush=True)
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = True
    for name in (sys.argv[1:] or list(SHAPES)):
        run(name, dev)


if __name__ == "__main__":
    main()
