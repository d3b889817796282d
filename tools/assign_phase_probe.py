"""Calibration: k_lloyd1 back-to-back launch time (pcm_time_assign) after a given
number of iterations -- does the assign kernel run slower inside the iteration
loop because of its lists at that iteration, or because k_step runs between?
usage: python tools/assign_phase_probe.py"""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pcm_amd import lloyd
from pcm_amd.engine import Engine, synth_rows, synth_uniform
N, K, D = 100_000_000, 1024, 3
X = synth_uniform(N, D, seed=0)
C0 = synth_rows(np.sort(np.random.default_rng(1).choice(N, K, replace=False)), D, seed=0)
for it in (3, 13, 23, 43):
    eng = Engine(D, K, torch.float32, max_iter=200)
    lloyd.prepare(eng, X)
    eng.begin(C0, 0.0, 200)
    eng.iterate(it)
    eng.timing(True)
    eng.iterate(10)   # 10 more, interleaved with k_step, HIP events per launch
    tm = eng.timing_read()
    eng.timing(False)
    torch.cuda.synchronize()
    cand = eng.candidate_stats()
    ms = eng.time_assign(20)
    print(f"iterations {it:2d}-{it + 10:2d}: assign with k_step between (events) {tm['assign_ms'] * 1e3:6.1f} us; "
          f"then back to back {ms * 1e3:6.1f} us; lists mean {cand['mean']:.3f}", flush=True)
    del eng
    torch.cuda.empty_cache()
