"""Calibration (debug build -DPCM_DBG_TIMING): per-block phase times of the
fused k_step of the last of `iters` iterations.  usage:
python tools/step_timing2.py SO_PATH [iters] [N K D]  (default config 3)"""
import ctypes, os, sys
import numpy as np
os.environ["PCM_SO"] = sys.argv[1]
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pcm_amd import lloyd, _lib
from pcm_amd.engine import Engine, synth_rows, synth_uniform
N, K, D = (int(v) for v in sys.argv[3:6]) if len(sys.argv) > 5 else (100_000_000, 1024, 3)
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
X = synth_uniform(N, D, seed=0, start=0)
C0 = synth_rows(np.sort(np.random.default_rng(1).choice(N, K, replace=False)), D, seed=0)
eng = Engine(D, K, torch.float32, max_iter=50)
lloyd.prepare(eng, X, None)
eng.begin(C0, 0.0, 50)
eng.iterate(iters); torch.cuda.synchronize()
st = eng.status()
lib = _lib.load()
lib.pcm_debug_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
nb = 8192
buf = np.zeros((nb, 16), np.uint64)
assert lib.pcm_debug_timing(buf.ctypes.data_as(ctypes.c_void_p), nb) == 0
t = buf.astype(np.int64)
nbk = int((t[:, 0] > 0).sum())
t = t[:nbk]
t0 = t[:, 0].min()
us = lambda v: v / 100.0   # s_memrealtime: 100 MHz
print(f"iters {st['iter']} rebuilds {st['list_rebuilds']} blocks {nbk}")
print("block start spread us: p50 %.1f p90 %.1f max %.1f" % tuple(us(np.percentile(t[:, 0] - t0, q)) for q in (50, 90, 100)))
w = t
print("centres+drift us (start->6): p50 %.1f max %.1f" % (us(np.median(w[:, 6] - w[:, 0])), us((w[:, 6] - w[:, 0]).max())))
print("body us (6->3): p50 %.1f max %.1f" % (us(np.median(w[:, 3] - w[:, 6])), us((w[:, 3] - w[:, 6]).max())))
c = t
for k0, k1, name in ((6, 4, "coarse reference"), (4, 5, "coarse prune"), (5, 1, "coarse compact"), (1, 2, "children")):
    ok = (c[:, k0] > 0) & (c[:, k1] > 0)
    if ok.any():
        dd = c[ok, k1] - c[ok, k0]
        print("%s us: p50 %.1f max %.1f" % (name, us(np.median(dd)), us(dd.max())))
print("end of bodies (rel. first start) us: p50 %.1f max %.1f" % (us(np.median(t[:, 3] - t0)), us(t[:, 3].max() - t0)))
last = t[:, 7].max()
print("last block finished at %.1f us" % us(last - t0))
ok = (c[:, 1] > 0) & (c[:, 2] > 0)
ch = us(c[ok, 2] - c[ok, 1]); mp = c[ok, 8]; bid = np.nonzero(ok)[0]
o = np.argsort(-ch)[:8]
print("slowest children blocks (block, us, coarse-list length):", [(int(bid[i]), round(float(ch[i]), 1), int(mp[i])) for i in o])
print("coarse-list length p10/p50/p90/max:", [int(np.percentile(mp, q)) for q in (10, 50, 90, 100)])
for k0, k1, name in ((1, 10, "pair 0 (boxes)"), (10, 11, "pair A (refs)"), (11, 12, "pair B (prune)"), (12, 2, "pair C (write)")):
    ok = (c[:, k0] > 0) & (c[:, k1] > 0)
    if ok.any():
        dd = c[ok, k1] - c[ok, k0]
        print("%s us: p50 %.2f max %.2f (%d blocks)" % (name, us(np.median(dd)), us(dd.max()), ok.sum()))
