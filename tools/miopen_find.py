"""Populate MIOpen's user find-db for every convolution of the cfg-2 forward (live-region
regulariser included): one MVSNet.forward with torch.backends.cudnn.benchmark = True (exhaustive
MIOpen find), then the db files are left in $MIOPEN_USER_DB_PATH for tools/miopen_db.

Usage (GPU box): MIOPEN_USER_DB_PATH=gpurun_out/miopen_db python tools/miopen_find.py
"""
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402


def heartbeat():
    t0 = time.time()
    while True:
        time.sleep(30)
        print("... find running %.0f s" % (time.time() - t0), flush=True)


def main():
    threading.Thread(target=heartbeat, daemon=True).start()
    print("db", os.environ.get("MIOPEN_USER_DB_PATH"), flush=True)
    dev = torch.device("cuda", 0)
    B, V, D, H, W = 4, 3, 192, 512, 640
    net = bench.build_model(D, H, W, dev)
    inputs = bench.make_inputs(B, V, H, W, 0, dev)
    torch.backends.cudnn.benchmark = True
    with torch.no_grad():
        for i in range(2):
            t = time.time()
            net(*inputs, B, V)
            torch.cuda.synchronize()
            print("step %d %.1f s" % (i, time.time() - t), flush=True)
    torch.backends.cudnn.benchmark = False
    with torch.no_grad():
        t = time.time()
        for _ in range(5):
            net(*inputs, B, V)
        torch.cuda.synchronize()
    print("step with db, benchmark off: %.2f ms" % ((time.time() - t) / 5 * 1000), flush=True)


if __name__ == "__main__":
    main()
