"""Calibration (debug build -DPCM_DBG_TIMING): per-phase times of the last
k_kpp_search launch of a k-means++ seeding.  usage: python tools/kpp_timing.py SO [N K D]"""
import ctypes, os, sys
import numpy as np
os.environ["PCM_SO"] = sys.argv[1]
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcm_amd
from pcm_amd import _lib
from pcm_amd.engine import synth_uniform
n, k, d = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (100_000_000, 1024, 3)
X = synth_uniform(n, d, seed=0)
pcm_amd.kmeans_plusplus(X, k, random_state=0)
torch.cuda.synchronize()
lib = _lib.load()
lib.pcm_debug_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros((8192, 16), np.uint64)
assert lib.pcm_debug_timing(buf.ctypes.data_as(ctypes.c_void_p), 8192) == 0
t = buf.astype(np.int64)
L = 2 + int(np.log(k))
us = lambda v: v / 100.0
t0 = t[:L + 64, 0].min()
print("search blocks (phase ends, us after the first block start):")
for b in range(L):
    r = t[b]
    print(b, " ".join(f"{j}:{us(r[j] - t0):6.2f}" for j in (0, 2, 3, 4, 5, 6, 7) if r[j] > 0), " loc", int(r[9]), "l2", int(r[10]))
g = t[L:L + 64]
print("gmax blocks: start p50 %.2f max %.2f  end p50 %.2f max %.2f" % (us(np.median(g[:, 0] - t0)), us((g[:, 0] - t0).max()),
                                                                   us(np.median(g[:, 8] - t0)), us((g[:, 8] - t0).max())))
# last k_kpp_eval launch (c = k - 1): per-block phase stamps (DBG_E) and reached cells of wave 0
lib.pcm_debug_timing_eval.argtypes = [ctypes.c_void_p, ctypes.c_int]
ev = np.zeros((8192, 8), np.uint64)
assert lib.pcm_debug_timing_eval(ev.ctypes.data_as(ctypes.c_void_p), 8192) == 0
e = ev.astype(np.int64)
nb = int((e[:, 0] > 0).sum())
e = e[:nb]
# the stamp table keeps blocks of earlier (larger-grid) launches: keep the blocks
# that started within 300 us of the latest start (the last launch)
e = e[e[:, 0] >= e[:, 0].max() - 30000]
nb = len(e)
t0 = e[:, 0].min()
print(f"eval blocks {nb}: items total {int(e[0, 5])}; reached cells of wave 0 p50 {np.median(e[:, 4]):.0f} max {e[:, 4].max()}")
for k, name in ((0, "start"), (1, "setup"), (3, "reach tests"), (6, "first cell"), (2, "cells done"), (7, "end")):
    if not (e[:, k] > 0).any():
        continue
    v = (e[e[:, k] > 0, k] - t0) / 100.0
    print(f"  {name:10s} us after first start: p50 {np.median(v):6.2f} p90 {np.percentile(v, 90):6.2f} max {v.max():6.2f}")
