"""Diff one engine E-step + accumulation (labels, counts, sums) against the oracle."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcm_amd  # noqa: E402
from pcm_amd.engine import Engine  # noqa: E402
from pcm_amd.fixed import fixed_q  # noqa: E402
from oracle import lloyd_ref as R  # noqa: E402


def check(X, C, label):
    n, d = X.shape
    k = C.shape[0]
    eng = Engine(d, k, torch.float32, max_iter=4)
    Xt = torch.from_numpy(X).cuda()
    _, _, mx = eng.bbox(Xt)
    q = fixed_q(mx)
    eng.build(Xt, q, 0)
    eng.begin(torch.from_numpy(C).cuda(), 0.0, 4)
    eng.iter_local()
    torch.cuda.synchronize()
    st = eng.stats.cpu().numpy()
    lab = eng.labels().cpu().numpy()
    rl, rs, rc, rch = R.local_stats(X, C, np.full(n, -1, np.int32), np.asarray(q, np.int32))
    sums = st[: k * (d + 1)].reshape(k, d + 1)
    print(label, "info", eng.layout_info(), eng.candidate_stats())
    print("  labels diff:", int((lab != rl).sum()), " counts diff:", int((sums[:, d] != rc).sum()),
          " sums diff:", int((sums[:, :d] != rs).sum()), " changed:", int(st[-1]), rch)
    import ctypes
    lib = eng.lib
    lib.pcm_debug_layout.argtypes = [ctypes.c_void_p] * 5
    xs = torch.empty(d * (((n + 3) // 4) * 4 + 4), dtype=torch.float32, device="cuda")
    ls = torch.empty(n, dtype=torch.int32, device="cuda")
    pm = torch.empty(n, dtype=torch.int32, device="cuda")
    rc_ = lib.pcm_debug_layout(eng.h, ctypes.c_void_p(xs.data_ptr()), ctypes.c_void_p(ls.data_ptr()),
                               ctypes.c_void_p(pm.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    npad = ((n + 3) // 4) * 4 + 4
    xs = xs.cpu().numpy().reshape(npad // 4, d, 4).transpose(0, 2, 1).reshape(npad, d)[:n]   # AoSoA-4
    ls = ls.cpu().numpy()
    pm = pm.cpu().numpy().astype(np.int64)
    print("  debug rc", rc_, "perm is permutation:", np.array_equal(np.sort(pm), np.arange(n)),
          " xs == X[perm]:", np.array_equal(xs, X[pm]))
    ref_sorted = R.assign(np.ascontiguousarray(xs), C)
    bad = np.flatnonzero(ls != ref_sorted)
    print("  sorted-order label diff:", bad.size, "first", bad[:10])
    if bad.size:
        i = bad[0]
        dd = R.sqdist(np.ascontiguousarray(xs[i:i + 1]), C)[0]
        print("   row", i, "x", xs[i], "gpu", ls[i], "ref", ref_sorted[i], "d_gpu", dd[ls[i]], "d_ref", dd[ref_sorted[i]])
        print("   labels around:", ls[max(0, i - 6):i + 6], ref_sorted[max(0, i - 6):i + 6])
    eng.final()
    torch.cuda.synchronize()
    lab1 = eng.labels().cpu().numpy()
    print("  final-mode labels diff:", int((lab1 != rl).sum()))
    bad = np.flatnonzero(sums[:, d] != rc)[:5]
    for j in bad:
        print("   cluster", j, "gpu cnt", sums[j, d], "ref", rc[j], "gpu sum", sums[j, :d], "ref", rs[j])
    bad = np.flatnonzero((sums[:, :d] != rs).any(1))[:5]
    for j in bad:
        print("   sumdiff cluster", j, sums[j, :d] - rs[j], "cnt", rc[j])


if __name__ == "__main__":
    g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "cfg1_n10k_k8.npz"))
    check(g["X"], g["C0"], "cfg1")
    X = R.splitmix_uniform(200_000, 3, 2)
    check(X, X[R.init_indices(200_000, 1024)], "200k/1024")
    X = R.splitmix_uniform(100_000, 3, 1)
    check(X, X[R.init_indices(100_000, 64)], "100k/64")
