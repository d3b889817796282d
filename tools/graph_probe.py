"""Calibration: per-iteration wall time of eager launches vs one captured HIP graph."""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcm_amd
from pcm_amd import lloyd
from pcm_amd.engine import Engine, synth_rows, synth_uniform
N, K, D = 100_000_000, 1024, 3
X = synth_uniform(N, D, seed=0, start=0)
C0 = synth_rows(np.sort(np.random.default_rng(1).choice(N, K, replace=False)), D, seed=0)
eng = Engine(D, K, torch.float32, max_iter=200)
lloyd.prepare(eng, X, None)
eng.begin(C0, 0.0, 200)
eng.iterate(3); torch.cuda.synchronize()
s = torch.cuda.Stream()
g = torch.cuda.CUDAGraph()
def eager():
    t0 = time.perf_counter(); eng.iterate(20); torch.cuda.synchronize(); return (time.perf_counter() - t0) / 20
def graph():
    t0 = time.perf_counter(); g.replay(); torch.cuda.synchronize(); return (time.perf_counter() - t0) / 20
te1 = eager()
with torch.cuda.graph(g, stream=s):
    eng.iterate(20)
torch.cuda.synchronize()
it0 = eng.status()["iter"]
tg1 = graph(); te2 = eager(); tg2 = graph(); te3 = eager()
print(f"from iter {it0}: eager {te1*1e6:.1f} | graph {tg1*1e6:.1f} | eager {te2*1e6:.1f} | graph {tg2*1e6:.1f} | eager {te3*1e6:.1f} us/iter; end iter {eng.status()['iter']}")
