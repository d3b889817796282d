"""Calibration (debug build with -DPCM_DBG_TIMING): per-block phase times of k_step."""
import ctypes, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcm_amd
from pcm_amd import lloyd, _lib
from pcm_amd.engine import Engine, synth_rows, synth_uniform
N, K, D = 100_000_000, 1024, 3
X = synth_uniform(N, D, seed=0, start=0)
C0 = synth_rows(np.sort(np.random.default_rng(1).choice(N, K, replace=False)), D, seed=0)
eng = Engine(D, K, torch.float32, max_iter=50)
lloyd.prepare(eng, X, None)
eng.begin(C0, 0.0, 50)
eng.iterate(10); torch.cuda.synchronize()
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
buf = np.zeros((nb, 8), np.uint64)
lib = _lib.load()
lib.pcm_debug_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
assert lib.pcm_debug_timing(buf.ctypes.data_as(ctypes.c_void_p), nb) == 0
t = buf.astype(np.int64)
t0 = t[:, 0].min()
us = lambda v: v / 100.0   # s_memrealtime: 100 MHz
print("block start spread (us): p50 %.1f p90 %.1f max %.1f" % tuple(us(np.percentile(t[:, 0] - t0, q)) for q in (50, 90, 100)))
print("phase0 (stats->LDS) us: p50 %.1f max %.1f" % (us(np.median(t[:, 3] - t[:, 0])), us((t[:, 3] - t[:, 0]).max())))
print("coarse us: p50 %.1f max %.1f" % (us(np.median(t[:, 1] - t[:, 3])), us((t[:, 1] - t[:, 3]).max())))
c = t[:-1]
print("  coarse split p50 us: ref-search %.1f | prune %.1f | compaction %.1f" % (us(np.median(c[:, 4] - c[:, 3])), us(np.median(c[:, 5] - c[:, 4])), us(np.median(c[:, 1] - c[:, 5]))))
print("children us: p50 %.1f max %.1f" % (us(np.median(t[:, 2] - t[:, 1])), us((t[:, 2] - t[:, 1]).max())))
nbk = int((t[:, 0] > 0).sum())
print("blocks", nbk, "; kernel span (first start -> last cand end) us: %.1f" % us(t[:nbk, 2].max() - t0))
