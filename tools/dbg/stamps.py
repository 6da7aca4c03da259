"""Analyse cv_head s_memtime stamps (build with -DMVS_HEAD_STAMP, run with MVS_HEAD_STAMPS=<file>).

Per workgroup (first 512), per wave, stamp index: 0 start, then per prologue phase, then per step k:
7 + 3k work A done (producer: items; consumer: conv_0_0), 8 + 3k work B done (producer: coords;
consumer: conv_1_0), 9 + 3k barrier passed."""
import sys
import numpy as np
KWG, KN = 512, 128
raw = np.fromfile(sys.argv[1], dtype=np.uint64)
n = KWG * 8 * KN
runs = raw.size // n
st = raw[(runs - 1) * n:runs * n].reshape(KWG, 8, KN).astype(np.int64)
ok = (st[:, :, 9] > 0).all(1)
st = st[ok]
print("runs in file", runs, "workgroups with stamps", st.shape[0])
nst = int((st[0, 0] > 0).sum())
ksteps = (nst - 7) // 3
print("stamps per wave", nst, "steps", ksteps)
t0 = st[:, :, 0].min(1, keepdims=True)
rel = st - t0[:, :, None]
P, C = slice(4, 8), slice(0, 4)
pro_total = rel[:, :, 6].mean()
print("prologue end (barrier 3 passed): %.0f ticks" % pro_total)
for name, sl in (("producer", P), ("consumer", C)):
    a = rel[:, sl]
    for k in range(min(ksteps, 6)):
        base = a[:, :, 6 + 3 * k]
        wa = (a[:, :, 7 + 3 * k] - base).mean()
        wb = (a[:, :, 8 + 3 * k] - a[:, :, 7 + 3 * k]).mean()
        bw = (a[:, :, 9 + 3 * k] - a[:, :, 8 + 3 * k]).mean()
        print("%s step %d: A %.0f B %.0f barrier-wait %.0f" % (name, k, wa, wb, bw))
    ks = range(1, ksteps)
    wa = np.mean([(a[:, :, 7 + 3 * k] - a[:, :, 6 + 3 * k]).mean() for k in ks])
    wb = np.mean([(a[:, :, 8 + 3 * k] - a[:, :, 7 + 3 * k]).mean() for k in ks])
    bw = np.mean([(a[:, :, 9 + 3 * k] - a[:, :, 8 + 3 * k]).mean() for k in ks])
    mx = np.mean([(a[:, :, 8 + 3 * k] - a[:, :, 6 + 3 * k]).max(1).mean() for k in ks])
    print("%s steps 1..: A %.0f  B %.0f  barrier-wait %.0f  (slowest wave's A+B %.0f)" % (name, wa, wb, bw, mx))
step = np.mean([(rel[:, :, 9 + 3 * k] - rel[:, :, 6 + 3 * k]).mean() for k in range(1, ksteps)])
print("step (barrier to barrier) %.0f ticks; whole WG %.0f ticks" % (step, rel[:, :, 6 + 3 * ksteps].max(1).mean()))
