"""CPU restatement of the dense (generic-D) Lloyd path, SURVEY.md §8 row a9.

TEST INFRASTRUCTURE ONLY (same rules as ``oracle/lloyd_ref.py``): only
``tests/`` may import it, as the checker; the product path never does.

The reference's only executed K-means is
``KMeans(n_clusters=5, random_state=42, n_init=10).fit_predict(StandardScaler(X))``
on ~1500 x 20 float64 superpixel features
(``members/jasraj/land_use_classification/core.py:225-228``).  This module
restates scikit-learn 1.7.2's ``_kmeans_single_lloyd`` (``sklearn/cluster/_kmeans.py:623-752``)
for any number of features, in the INPUT precision (float64 stays float64, as
in scikit-learn), with the canonical arithmetic of ``csrc/pcm_dense.hip``:

* distance: ``sum_a (x_a - c_a)**2`` accumulated feature by feature in the
  input dtype (scikit-learn's GEMM form ``||c||^2 - 2 x.c``,
  ``_k_means_lloyd.pyx:196-203``, differs only on near-ties at the 1e-16 level);
  argmin strict ``<`` in centroid order (``:205-213``);
* sums: exact int64 fixed point ``trunc(ldexp(x_a, q_a))``,
  ``q_a = 62 - e_a - bitlen(n)`` with ``max|x_a| < 2**e_a``;
* centre: ``dtype((float64(S) * 2**-q) * (1.0 / count))`` (``_average_centers``
  multiplies by ``alpha = 1 / weight``, ``_k_means_common.pyx:274-295``);
* empty clusters: the farthest points (distance desc, row asc) move into the
  empty clusters (fixed list, ``_k_means_common.pyx:167-211``); a cluster still
  empty copies the averaged centre of the first largest one;
* shift: per centre ``sqrt`` of ``_euclidean_dense_dense``'s sum (features in
  groups of 4, ``_k_means_common.pyx:17-43``), total = sequential sum of the
  squares (``_kmeans.py:724-732``); stop on unchanged labels or shift <= tol;
* inertia: ``ldexp(float(sum_i trunc(d_i * 2**s)), -s)`` (exact integer sum).

Pinned against scikit-learn golden runs (``tests/golden/make_golden.py``,
``jasraj_*.npz``): labels and ``n_iter`` equal, centres within 1e-12
(float64), inertia within 1e-12.
"""
from __future__ import annotations

import math

import numpy as np


def points(X) -> np.ndarray:
    X = np.asarray(X)
    if X.dtype not in (np.float32, np.float64):
        X = X.astype(np.float64)
    return np.ascontiguousarray(X)


def fixed_q(maxabs, n: int) -> np.ndarray:
    nb = int(n).bit_length()
    out = []
    for m in np.asarray(maxabs, dtype=np.float64):
        e = 0 if m == 0.0 else math.frexp(float(m))[1]
        out.append(62 - e - nb)
    return np.asarray(out, dtype=np.int64)


def inertia_scale(maxabs) -> int:
    bound = 0.0
    for m in np.asarray(maxabs, dtype=np.float64):
        e = 0 if m == 0.0 else math.frexp(float(m))[1]
        bound += math.ldexp(1.0, 2 * (e + 1))
    _, eb = math.frexp(bound * (1.0 + 2.0 ** -20))
    return 64 - eb


def sqdist(X, C) -> np.ndarray:
    """(n, k) canonical distances in X's dtype, features accumulated in order."""
    acc = None
    for a in range(X.shape[1]):
        diff = X[:, None, a] - C[None, :, a]
        sq = diff * diff
        acc = sq if acc is None else acc + sq
    return acc


def assign(X, C):
    out = np.empty(X.shape[0], dtype=np.int32)
    dist = np.empty(X.shape[0], dtype=X.dtype)
    step = max(1, 1 << 20 // max(1, C.shape[0] * X.shape[1]))
    for s in range(0, X.shape[0], step):
        dd = sqdist(X[s:s + step], C)
        out[s:s + step] = np.argmin(dd, axis=1)
        dist[s:s + step] = dd[np.arange(dd.shape[0]), out[s:s + step]]
    return out, dist


def to_fixed(X, q) -> np.ndarray:
    return np.ldexp(X.astype(np.float64), q[None, :].astype(np.int32)).astype(np.int64)


def shift_total(Cn, Co) -> float:
    tot = 0.0
    d = Cn.shape[1]
    for j in range(Cn.shape[0]):
        res = 0.0
        a0 = 0
        while a0 + 4 <= d:
            g = None
            for a in range(a0, a0 + 4):
                df = float(Cn[j, a]) - float(Co[j, a])
                sq = df * df
                g = sq if g is None else g + sq
            res = res + g
            a0 += 4
        for a in range(a0, d):
            df = float(Cn[j, a]) - float(Co[j, a])
            res = res + df * df
        r = math.sqrt(res)
        tot = tot + r * r
    return tot


def inertia_exact(d, s: int) -> float:
    w = np.ldexp(np.asarray(d).astype(np.float64), s)
    if w.size and float(w.max()) >= 2.0 ** 64:
        return math.inf
    w = w.astype(np.uint64)
    lo = int(np.sum(w & np.uint64(0xFFFFFFFF), dtype=np.uint64))
    hi = int(np.sum(w >> np.uint64(32), dtype=np.uint64))
    return math.ldexp(float(lo + (hi << 32)), -s)


def dense_fit(X, C0, max_iter: int = 300, tol: float = 0.0):
    """``_kmeans_single_lloyd`` restated for the dense path; returns dict(labels,
    centers, inertia, n_iter, strict, changed, shift)."""
    X = points(X)
    T = X.dtype
    C = np.ascontiguousarray(np.asarray(C0, dtype=T))
    n, d = X.shape
    k = C.shape[0]
    maxabs = np.abs(X).max(axis=0).astype(np.float64)
    q = fixed_q(maxabs, n)
    xq = to_fixed(X, q)
    scale = np.ldexp(1.0, -q)
    labels_old = np.full(n, -1, np.int32)
    strict = False
    changed, shifts = [], []
    it = 0
    for it in range(max_iter):
        labels, dist = assign(X, C)
        nch = int(np.count_nonzero(labels != labels_old))
        counts = np.bincount(labels, minlength=k).astype(np.int64)
        sums = np.zeros((k, d), dtype=np.int64)
        np.add.at(sums, labels, xq)
        empty = np.flatnonzero(counts == 0)
        if empty.size:
            order = np.lexsort((np.arange(n), -dist.astype(np.float64)))
            if float(dist[order[0]]) > 0.0:
                for t, j in enumerate(empty[:n]):
                    p = order[t]
                    old = labels[p]
                    sums[old] -= xq[p]
                    counts[old] -= 1
                    sums[j] = xq[p]
                    counts[j] = 1
        Cn = C.copy()
        nz = counts > 0
        arg = int(np.argmax(counts))
        for j in range(k):
            src = j if (nz[j] or not nz.any()) else arg
            if counts[src] > 0:
                Cn[j] = ((sums[src].astype(np.float64) * scale) * (1.0 / float(counts[src]))).astype(T)
        sh = shift_total(Cn, C)
        changed.append(nch)
        shifts.append(sh)
        C = Cn
        if nch == 0:
            strict = True
            break
        if sh <= tol:
            break
        labels_old = labels
    labels, dist = assign(X, C)
    return dict(labels=labels, centers=C, inertia=inertia_exact(dist, inertia_scale(maxabs)), n_iter=it + 1,
                strict=strict, changed=changed, shift=shifts)
