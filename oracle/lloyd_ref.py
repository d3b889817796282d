"""CPU restatement of the canonical multi-day point-cloud Lloyd step.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker.  The product path (``pcm_amd``) never imports it and has no CPU
fallback.

What this restates
------------------
The reference repository has no K-means of its own: the only
K-means it executes is scikit-learn's Lloyd, called from
``members/jasraj/land_use_classification/core.py:227-228``.  This module restates
that algorithm (scikit-learn 1.7.2, installed in the build container):

* ``sklearn/cluster/_kmeans.py:623-752``  ``_kmeans_single_lloyd`` (driver loop,
  strict-label and shift-tolerance convergence, final E-step, inertia);
* ``sklearn/cluster/_k_means_lloyd.pyx:23-165`` ``lloyd_iter_chunked_dense`` and
  ``:168-218`` ``_update_chunk_dense`` (E-step argmin with strict ``<`` so the
  lowest index wins, per-cluster weight and coordinate sums);
* ``sklearn/cluster/_k_means_common.pyx:167-211`` ``_relocate_empty_clusters_dense``,
  ``:274-295`` ``_average_centers``, ``:298-311`` ``_center_shift``.

with the canonical arithmetic fixed by this build
so that labels can be bit-exact between CPU and GPU:

* distance: ``((d0*d0 + d1*d1) + d2*d2) + d3*d3`` with ``d_a = x_a - c_a``,
  every operation an IEEE float32 operation (no FMA); fp16 inputs are widened
  exactly, float64 inputs are rounded to float32 at the boundary;
  (sklearn evaluates ``||c||^2 - 2 x.c`` through a GEMM, ``_k_means_lloyd.pyx:196-203``,
  which differs from the direct form on ~1e-5 of near-tie labels);
* argmin: strict ``<`` scanning centroids in index order (``:205-213``);
* accumulation: exact int64 fixed point, ``xq = trunc(ldexp(x, q_a))`` (exact
  power-of-two scaling, truncation toward zero) with a per-dimension
  ``q_a = QBITS - e_a`` where ``max|x_a| < 2**e_a``; the result is independent
  of summation order, block order and GPU count;
* update: ``c = float32(float64(S) * 2**-q / float64(count))``;
* empty clusters: sklearn's farthest-point relocation with a deterministic
  order (distance descending, then global point index ascending); a cluster
  still empty afterwards copies the (averaged) centre of the first
  largest cluster;
* shift: ``sum_j sum_a (c_new - c_old)**2`` in float64 with the fixed reduction
  tree of the GPU finalize kernel (1024 sequential lanes, then halving);
* inertia (``_kmeans.py:750``, sklearn's ``_inertia_dense``): the exact integer
  ``sum_i trunc(d_i * 2**s)`` of the canonical float32 distances, ``s`` from the
  global fixed-point exponents (``inertia_scale``), converted to float64 once
  and scaled by ``2**-s`` -- independent of summation order, block count and
  world size (sklearn's float32/float64 sum depends on its thread count).

Parity status: pinned against scikit-learn golden vectors generated in the
build container (``tests/golden/make_golden.py``) and against the
hand-computed sklearn known-answer tests restated as numbers in
``tests/test_oracle_golden.py``.
"""
from __future__ import annotations

import math

import numpy as np

QBITS = 25          # |xq| < 2**QBITS; GPU lanes hold per-lane partial sums in int32
CHUNK = 8192        # rows per distance block (memory bound only)
SHIFT_LANES = 1024  # lanes of the GPU finalize reduction tree


# ---------------------------------------------------------------- inputs
def as_f32_points(X) -> np.ndarray:
    """Boundary cast: fp16 widens exactly, fp64 rounds to nearest fp32."""
    X = np.asarray(X)
    if X.ndim != 2:
        raise ValueError("points must be a 2-D (N, D) array")
    if X.dtype != np.float32:
        X = X.astype(np.float32)
    return np.ascontiguousarray(X)


def splitmix_uniform(n: int, d: int, seed: int, start: int = 0) -> np.ndarray:
    """Counter-based U[0,1) float32 cloud, identical to the device generator.

    Element ``(i, a)`` uses counter ``(start+i)*d + a``; value is the top 24 bits
    of splitmix64(seed-mixed counter) times 2**-24 (exactly representable).
    """
    with np.errstate(over="ignore"):
        ctr = np.arange((start) * d, (start + n) * d, dtype=np.uint64)
        z = (np.uint64(seed) * np.uint64(0xD1B54A32D192ED03)
             + (ctr + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    v = (z >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)
    return v.reshape(n, d)


def init_indices(n: int, k: int, seed: int = 1) -> np.ndarray:
    """SURVEY.md §8d init: sorted ``default_rng(seed).choice(n, k, replace=False)``."""
    return np.sort(np.random.default_rng(seed).choice(n, k, replace=False))


# ---------------------------------------------------------------- E-step
def sqdist(X: np.ndarray, C: np.ndarray) -> np.ndarray:
    """Canonical float32 squared distances, shape (n, k)."""
    acc = None
    for a in range(X.shape[1]):
        diff = X[:, None, a] - C[None, :, a]
        sq = diff * diff
        acc = sq if acc is None else acc + sq
    return acc


def sqdist_rows(X: np.ndarray, Crow: np.ndarray) -> np.ndarray:
    """Canonical float32 distance of each row of X to the matching row of Crow."""
    acc = None
    for a in range(X.shape[1]):
        diff = X[:, a] - Crow[:, a]
        sq = diff * diff
        acc = sq if acc is None else acc + sq
    return acc


def assign(X: np.ndarray, C: np.ndarray) -> np.ndarray:
    """Nearest centroid, lowest index wins ties (``_k_means_lloyd.pyx:205-213``)."""
    n = X.shape[0]
    out = np.empty(n, dtype=np.int32)
    step = max(1, CHUNK * 64 // max(1, C.shape[0]))
    for s in range(0, n, step):
        out[s:s + step] = np.argmin(sqdist(X[s:s + step], C), axis=1)
    return out


# ---------------------------------------------------------------- fixed point
def fixed_q(X: np.ndarray) -> np.ndarray:
    """Per-dimension fixed-point exponent q_a with |trunc(ldexp(x, q_a))| < 2**QBITS."""
    maxabs = np.max(np.abs(X), axis=0).astype(np.float64) if X.shape[0] else np.zeros(X.shape[1])
    _, e = np.frexp(maxabs)
    e = np.where(maxabs == 0, 0, e)
    return (QBITS - e).astype(np.int32)


def to_fixed(X: np.ndarray, q: np.ndarray) -> np.ndarray:
    return np.ldexp(X, q.astype(np.int32)[None, :]).astype(np.int64)   # truncates toward zero


def segment_sums(labels: np.ndarray, vals: np.ndarray, k: int) -> np.ndarray:
    """Exact int64 per-label sums of int64 rows (order independent)."""
    out = np.zeros((k, vals.shape[1]), dtype=np.int64)
    if labels.size == 0:
        return out
    order = np.argsort(labels, kind="stable")
    sl = labels[order]
    starts = np.flatnonzero(np.r_[True, sl[1:] != sl[:-1]])
    red = np.add.reduceat(vals[order], starts, axis=0)
    out[sl[starts]] = red
    return out


# ---------------------------------------------------------------- M-step
def local_stats(X, C, labels_old, q, weights=None, fast=False):
    """Per-shard E-step + accumulation: what one GPU rank contributes.

    ``fast`` uses the bit-identical C restatement (oracle/lloyd_ref.c)."""
    k = C.shape[0]
    if fast and weights is None:
        from . import cref
        return cref.lloyd_stats(X, C, q, labels_old)
    labels = assign(X, C)
    n_changed = int(np.count_nonzero(labels != labels_old))
    xq = to_fixed(X, q)
    w = np.ones(X.shape[0], dtype=np.int64) if weights is None else np.asarray(weights, dtype=np.int64)
    counts = np.zeros(k, dtype=np.int64)
    np.add.at(counts, labels, w)
    sums = segment_sums(labels, xq * w[:, None], k)
    return labels, sums, counts, n_changed


def far_candidates(X, C, labels, gidx0: int, m: int, weights=None):
    """Local relocation candidates: the m points farthest from their centre.

    Returns (dist, global_index, label, xq-row-source X row) sorted by
    (dist desc, global index asc).  ``_k_means_common.pyx:185-187``.
    """
    dist = sqdist_rows(X, C[labels])
    # gidx0: the global row of local row 0 (row shard), or every local row's global row (spatial shard)
    gidx = np.asarray(gidx0, np.int64) if np.ndim(gidx0) else np.arange(X.shape[0], dtype=np.int64) + gidx0
    order = np.lexsort((gidx, -dist.astype(np.float64)))[:m]
    w = np.ones(X.shape[0], dtype=np.int64) if weights is None else np.asarray(weights, dtype=np.int64)
    return dist[order], gidx[order], labels[order], X[order], w[order]


def relocate(sums, counts, cand, q):
    """Apply sklearn's relocation (``_k_means_common.pyx:167-211``) to global stats.

    ``cand`` = merged candidate tuple (dist, gidx, label, Xrow, w) over all shards.
    Mutates sums/counts in place; returns number of relocated clusters.
    """
    empty = np.flatnonzero(counts == 0)
    n_empty = empty.size
    if n_empty == 0:
        return 0
    dist, gidx, lab, xr, w = cand
    order = np.lexsort((gidx, -dist.astype(np.float64)))
    dist, gidx, lab, xr, w = dist[order], gidx[order], lab[order], xr[order], w[order]
    if dist.size == 0 or float(dist.max()) == 0.0:
        return 0   # sklearn: "more clusters than non-duplicate samples"
    xq = to_fixed(xr, q)
    for i in range(n_empty):
        new, old = int(empty[i]), int(lab[i])
        sums[old] -= xq[i] * w[i]
        counts[old] -= w[i]
        sums[new] = xq[i] * w[i]
        counts[new] = w[i]
    return n_empty


def average(sums, counts, q, C_old):
    """``_average_centers`` with exact fixed-point sums."""
    k, d = sums.shape
    Cn = np.empty((k, d), dtype=np.float32)
    nz = counts > 0
    scale = np.ldexp(1.0, -q.astype(np.int64))
    Cn[nz] = ((sums[nz].astype(np.float64) * scale[None, :]) /
              counts[nz, None].astype(np.float64)).astype(np.float32)
    if (~nz).any():
        if nz.any():
            Cn[~nz] = Cn[int(np.argmax(counts))]
        else:
            Cn[~nz] = C_old[~nz]
    return Cn


def shift_total(Cn, Co) -> float:
    """Sum of squared centre shifts, fixed fp64 reduction tree of the finalize kernel."""
    k, d = Cn.shape
    diff = Cn.astype(np.float64) - Co.astype(np.float64)
    s = None
    for a in range(d):
        t = diff[:, a] * diff[:, a]
        s = t if s is None else s + t
    pad = (-k) % SHIFT_LANES
    s = np.concatenate([s, np.zeros(pad)]).reshape(-1, SHIFT_LANES)
    acc = s[0].copy()
    for r in range(1, s.shape[0]):
        acc = acc + s[r]
    while acc.size > 1:
        h = acc.size // 2
        acc = acc[:h] + acc[h:]
    return float(acc[0])


def inertia_scale(q) -> int:
    """Exponent s with trunc(d * 2**s) < 2**64 for every canonical distance d:
    |x_a|, |c_a| < 2**(QBITS - q_a) bound d by sum_a 4**(QBITS + 1 - q_a)
    (times 1 + 2**-20 for the float32 rounding)."""
    bound = sum(math.ldexp(1.0, 2 * (QBITS + 1 - int(qa))) for qa in q)
    _, e = math.frexp(bound * (1.0 + 2.0 ** -20))
    return 64 - e


def inertia_exact(d: np.ndarray, s: int) -> float:
    """``ldexp(float(sum trunc(d * 2**s)), -s)`` with the sum an exact integer."""
    w = np.ldexp(np.asarray(d, dtype=np.float32).astype(np.float64), s)
    if w.size and float(w.max()) >= 2.0 ** 64:
        return math.inf
    w = w.astype(np.uint64)
    lo = int(np.sum(w & np.uint64(0xFFFFFFFF), dtype=np.uint64))
    hi = int(np.sum(w >> np.uint64(32), dtype=np.uint64))
    return math.ldexp(float(lo + (hi << 32)), -s)


def inertia(X, C, labels, weights=None, q=None) -> float:
    d = sqdist_rows(X, C[labels])
    if weights is None:
        return inertia_exact(d, inertia_scale(fixed_q(X) if q is None else q))
    return float((d.astype(np.float64) * np.asarray(weights, dtype=np.float64)).sum())


# ---------------------------------------------------------------- driver
def assign_fast(X, C):
    from . import cref
    return cref.lloyd_stats(X, C, with_sums=False)[0]


def lloyd_fit(X, C0, max_iter=300, tol=0.0, weights=None, shards=1, history=False, fast=False):
    """``_kmeans_single_lloyd`` restated (``_kmeans.py:623-752``).

    ``tol`` is the absolute shift tolerance (sklearn's ``_tolerance`` output).
    ``shards`` splits rows into contiguous shards and reduces their integer
    stats, as the multi-GPU path does; results are identical for any value.
    Returns dict(labels, centers, inertia, n_iter, strict, changed, [history]).
    """
    X = as_f32_points(X)
    C = np.ascontiguousarray(np.asarray(C0, dtype=np.float32))
    n, d = X.shape
    k = C.shape[0]
    q = fixed_q(X)
    bounds = np.linspace(0, n, shards + 1).astype(np.int64)
    wt = None if weights is None else np.asarray(weights, dtype=np.int64)
    labels_old = np.full(n, -1, dtype=np.int32)
    strict = False
    changed, hist = [], []
    it = 0
    for it in range(max_iter):
        parts = []
        for r in range(shards):
            a, b = bounds[r], bounds[r + 1]
            parts.append(local_stats(X[a:b], C, labels_old[a:b], q,
                                     None if wt is None else wt[a:b], fast=fast))
        labels = np.concatenate([p[0] for p in parts])
        sums = sum(p[1] for p in parts)
        counts = sum(p[2] for p in parts)
        nch = sum(p[3] for p in parts)
        if (counts == 0).any():
            m = int((counts == 0).sum())
            cands = [far_candidates(X[bounds[r]:bounds[r + 1]], C, labels[bounds[r]:bounds[r + 1]],
                                    int(bounds[r]), m, None if wt is None else wt[bounds[r]:bounds[r + 1]])
                     for r in range(shards)]
            merged = tuple(np.concatenate([c[i] for c in cands]) for i in range(5))
            relocate(sums, counts, merged, q)
        Cn = average(sums, counts, q, C)
        shift = shift_total(Cn, C)
        changed.append(nch)
        if history:
            hist.append(dict(labels=labels.copy(), centers=Cn.copy(), sums=sums.copy(),
                             counts=counts.copy(), shift=shift))
        C = Cn
        if nch == 0:
            strict = True
            break
        if shift <= tol:
            break
        labels_old = labels
    labels = assign_fast(X, C) if fast else assign(X, C)
    out = dict(labels=labels, centers=C, inertia=inertia(X, C, labels, wt, q), n_iter=it + 1,
               strict=strict, changed=changed, q=q)
    if history:
        out["history"] = hist
    return out
