"""Calibration (debug build -DPCM_DBG_TIMING): per-step work of k-means++ eval and
apply -- cube items reach-tested and cells reached -- by seeding phase.
usage: python tools/kpp_counts.py SO [N K D]"""
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
lib = _lib.load()
lib.pcm_debug_kpp_counts.argtypes = [ctypes.c_void_p, ctypes.c_int]
zero = np.zeros((4096, 4), np.uint64)
pcm_amd.kmeans_plusplus(X, k, random_state=0)
torch.cuda.synchronize()
buf = np.zeros((4096, 4), np.uint64)
assert lib.pcm_debug_kpp_counts(buf.ctypes.data_as(ctypes.c_void_p), 4096) == 0
b = buf[1:k].astype(np.float64)
print(f"n={n} k={k} d={d}: per-step means (eval items tested, eval cells reached, apply items, apply reached)")
for lo, hi in ((0, 10), (10, 50), (50, 200), (200, 600), (600, k - 1)):
    r = b[lo:hi]
    print(f"  centres [{lo + 1}:{hi + 1}]  " + "  ".join(f"{v:12.0f}" for v in r.mean(axis=0)))
