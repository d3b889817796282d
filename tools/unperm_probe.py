"""Time pcm_labels (sorted-order labels -> row order) at N=100M after a short fit.
usage: PCM_UNPERM=<0|1|2> [PCM_UNPERM_WIN=rows] python tools/unperm_probe.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pcm_amd import lloyd  # noqa: E402
from pcm_amd.engine import Engine, synth_rows, synth_uniform  # noqa: E402

N, K, D = 100_000_000, 1024, 3
X = synth_uniform(N, D, seed=0)
C0 = synth_rows(np.sort(np.random.default_rng(1).choice(N, K, replace=False)), D, seed=0)
eng = Engine(D, K, torch.float32, max_iter=4)
lloyd.prepare(eng, X, lloyd.LOCAL)
lloyd.run(eng, C0, 4, 0.0, lloyd.LOCAL)
eng.final()
ref = eng.labels()
torch.cuda.synchronize()
ts = []
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out = eng.labels()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
    assert torch.equal(out, ref)
print(f"mode={os.environ.get('PCM_UNPERM', '0')} win={os.environ.get('PCM_UNPERM_WIN', '-')} labels ms: "
      + " ".join(f"{t:.3f}" for t in ts))
