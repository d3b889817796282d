"""Calibration (debug build -DPCM_DBG_TIMING): per-block phase times of the
k_lloyd launch of the last of `iters` iterations.
usage: python tools/lloyd_timing.py SO_PATH [iters] [N K D]  (default config 3)"""
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
lib = _lib.load()
lib.pcm_debug_timing_lloyd.argtypes = [ctypes.c_void_p, ctypes.c_int]
nb = 65536
buf = np.zeros((nb, 4), np.uint64)
assert lib.pcm_debug_timing_lloyd(buf.ctypes.data_as(ctypes.c_void_p), nb) == 0
t = buf.astype(np.int64)
t = t[t[:, 0] > 0]
t0 = t[:, 0].min()
us = lambda v: np.asarray(v) / 100.0   # s_memrealtime: 100 MHz
print(f"N={N} K={K} D={D} blocks {len(t)} kernel span {us(t[:, 3].max() - t0):.1f} us")
for name, a, b in (("start (rel. first)", None, 0), ("setup (start->first round)", 0, 1), ("rounds", 1, 2),
                   ("fold+exit", 2, 3), ("block total", 0, 3), ("end (rel. first start)", None, 3)):
    v = t[:, b] - (t0 if a is None else t[:, a])
    print("%-28s p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f us" % ((name,) + tuple(us(np.percentile(v, q)) for q in (10, 50, 90, 100))))
# concurrency: blocks resident over time (1 us bins)
span = int(us(t[:, 3].max() - t0)) + 1
occ = np.zeros(span + 1)
for s_, e_ in zip(us(t[:, 0] - t0).astype(int), us(t[:, 3] - t0).astype(int)):
    occ[s_:e_ + 1] += 1
print("resident blocks per us bin:", " ".join(str(int(x)) for x in occ[::max(1, span // 40)]))
