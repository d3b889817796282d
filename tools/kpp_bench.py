"""k-means++ timing on the synthetic bench cloud: python tools/kpp_bench.py N K D"""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcm_amd
from pcm_amd.engine import synth_uniform
n, k, d = (int(a) for a in sys.argv[1:4])
X = synth_uniform(n, d, seed=0)
pcm_amd.kmeans_plusplus(X[:10000].contiguous(), 8, random_state=0)   # warm-up (library, kernels)
for rep in range(2):   # the second call reuses torch's cached workspace
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    C, idx = pcm_amd.kmeans_plusplus(X, k, random_state=0)
    torch.cuda.synchronize()
    print(f"kmeans_plusplus n={n} k={k} d={d} call {rep}: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
