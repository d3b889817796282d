"""CPU restatement of the canonical k-means++ seeding.

TEST INFRASTRUCTURE ONLY (same rules as ``oracle/lloyd_ref.py``): only
``tests/`` may import it, as the checker; the product path never does.

Restates scikit-learn 1.7.2 ``_kmeans_plusplus`` (``sklearn/cluster/_kmeans.py:174-272``),
the default init of ``KMeans`` (``:1012-1019``) used at the reference's only
K-means call site (``members/jasraj/land_use_classification/core.py:227-228``):

* ``n_local_trials = 2 + int(log(k))`` (``:215-219``);
* first centre: ``random_state.choice(n, p=w / w.sum())`` (``:222``), i.e. one
  ``random_sample()`` searched (side='right') in the normalised float64 cdf
  (numpy ``RandomState.choice``); unit weights;
* each further centre (``:236-264``): ``L`` uniforms times the current
  potential are searched (side='left') in the cumulative sum of the
  closest-centre distances, clipped to ``n-1``; every candidate's potential is
  ``sum(min(closest, d(x, cand)))``; the first argmin wins and becomes the
  centre; ``closest`` is updated with it.

Canonical arithmetic fixed by this build so that CPU and GPU agree bit for bit
(sklearn sums float64 distances from a GEMM; this is where it can differ, on
near-boundary samples only):

* distance: the canonical float32 direct form of ``lloyd_ref.sqdist_rows``;
* weight of a point: ``w = trunc(ldexp(float64(d), s))`` as an unsigned 64-bit
  integer, with one scale ``s`` per cloud (``kpp_scale``) so that the sum over
  all points cannot overflow; potentials and cumulative sums are exact integers
  (any summation order gives the same value);
* a sample ``u`` (a double from ``random_sample``, an exact multiple of
  2**-53) selects the target ``floor(u * pot)`` computed exactly as
  ``(m * pot) >> 53`` with ``m = u * 2**53``.

Parity: pinned against ``sklearn.cluster.kmeans_plusplus`` (same seeds, same
random stream) on the cases of ``tests/test_kpp.py`` -- identical indices.  On
unstructured clouds a local trial whose potential ties another's within
sklearn's GEMM-form rounding can be chosen differently (uniform 20000 x 3,
K=64: 1 seed in 10); tests/test_estimator.py::test_unstructured_cloud_parity_limit.
"""
from __future__ import annotations

import math

import numpy as np

from .lloyd_ref import as_f32_points, sqdist_rows


def n_trials(k: int) -> int:
    return 2 + int(np.log(k))


def kpp_scale(n: int, maxd: float) -> int:
    """Exponent s with n * 2**s * maxd * (1 + 2**-20) < 2**62 (maxd: bound on any distance)."""
    if maxd <= 0 or n <= 0:
        return 0
    _, e = math.frexp(maxd * (1.0 + 2.0 ** -20))     # maxd' < 2**e
    nb = max(1, int(n - 1).bit_length())              # n <= 2**nb
    return int(62 - nb - e)


def max_dist_bound(X: np.ndarray) -> float:
    """Squared bbox diagonal (float64): bounds every canonical pairwise distance (+ rounding margin)."""
    if X.shape[0] == 0:
        return 0.0
    ext = X.max(axis=0).astype(np.float64) - X.min(axis=0).astype(np.float64)
    return float((ext * ext).sum())


def weights(d: np.ndarray, s: int) -> np.ndarray:
    return np.ldexp(d.astype(np.float64), s).astype(np.uint64)   # truncation (d >= 0)


def target(u: float, pot: int) -> int:
    m = int(round(u * 2.0 ** 53))
    assert m / 2.0 ** 53 == u
    return (m * int(pot)) >> 53


def first_index(n: int, u0: float, dtype=np.float32) -> int:
    """numpy RandomState.choice(n, p=w / w.sum()) given its one random_sample() draw,
    with sklearn's unit weights in X's dtype (``_check_sample_weight``)."""
    w = np.ones(n, dtype=dtype)
    p = (w / w.sum()).astype(np.float64)
    cdf = p.cumsum()
    cdf /= cdf[-1]
    return int(cdf.searchsorted(u0, side="right"))


def draws(seed, k: int, L: int):
    """The exact random stream sklearn's _kmeans_plusplus consumes (seed: int or RandomState)."""
    rs = seed if isinstance(seed, np.random.RandomState) else np.random.RandomState(seed)
    u0 = rs.random_sample()
    us = np.stack([rs.uniform(size=L) for _ in range(1, k)]) if k > 1 else np.zeros((0, L))
    return u0, us


def kmeanspp(X, k: int, seed, n_local_trials: int | None = None, keep_dtype: bool = False):
    """Returns (centers (k, d), indices (k,) int64).  Distances in float32 (the
    point-cloud path), or in X's own dtype when ``keep_dtype`` (the dense path,
    oracle/dense_ref.py: float64 features stay float64 as in scikit-learn)."""
    if keep_dtype:
        X = np.ascontiguousarray(np.asarray(X))
        if X.dtype not in (np.float32, np.float64):
            X = X.astype(np.float64)
    else:
        X = as_f32_points(X)
    n, d = X.shape
    L = n_trials(k) if n_local_trials is None else int(n_local_trials)
    u0, us = draws(seed, k, L)
    s = kpp_scale(n, max_dist_bound(X))
    idx = np.full(k, -1, dtype=np.int64)
    idx[0] = first_index(n, u0, X.dtype)
    closest = sqdist_rows(X, np.broadcast_to(X[idx[0]], X.shape))          # float32
    pot = int(weights(closest, s).sum(dtype=np.uint64))
    for c in range(1, k):
        cum = np.cumsum(weights(closest, s), dtype=np.uint64)
        tg = np.array([target(u, pot) for u in us[c - 1]], dtype=np.uint64)
        cand = np.minimum(np.searchsorted(cum, tg, side="left"), n - 1)
        best_pot, best_l, best_m = None, -1, None
        for l, ci in enumerate(cand):
            m = np.minimum(closest, sqdist_rows(X, np.broadcast_to(X[ci], X.shape)))
            pl = int(weights(m, s).sum(dtype=np.uint64))
            if best_pot is None or pl < best_pot:
                best_pot, best_l, best_m = pl, l, m
        idx[c] = cand[best_l]
        pot, closest = best_pot, best_m
    return X[idx].copy(), idx
