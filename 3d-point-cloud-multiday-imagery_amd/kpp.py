"""k-means++ seeding on the GPU.

``kmeans_plusplus`` mirrors ``sklearn.cluster.kmeans_plusplus`` (same
arguments, same ``(centers, indices)`` result, same random stream: a seeded
``RandomState`` yields the indices scikit-learn yields on the same cloud, up to
the canonical-arithmetic caveat of oracle/kpp_ref.py).  The host draws the
random numbers exactly as ``_kmeans_plusplus`` consumes them
(sklearn/cluster/_kmeans.py:215-248) and the HIP kernels of ``csrc/pcm_kpp.hpp``
do every pass over the cloud; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import _lib
from .engine import _ptr, _stream


def _scale(n: int, maxd: float) -> int:
    """Weight exponent: n * 2**s * maxd (with rounding margin) < 2**62 (computed
    again by pcm_kmeanspp from the device bounding box; kept for the tests)."""
    if maxd <= 0 or n <= 0:
        return 0
    _, e = math.frexp(maxd * (1.0 + 2.0 ** -20))
    return int(62 - max(1, int(n - 1).bit_length()) - e)


def _first_index(n: int, u0: float, weight_dtype=np.float32) -> int:
    """numpy RandomState.choice(n, p=w / w.sum()) for its single random_sample() draw u0,
    with sklearn's unit weights in X's dtype (``_check_sample_weight``).

    choice() searches u0 (side='right') in cdf = cumsum(p) / cumsum(p)[-1].
    float32 weights: p[i] = v (one float32 constant widened to float64); for
    n < 2**29 every partial sum (i + 1) * v is exact in float64 (v has 24
    significant bits), so cdf[i] = RN((i + 1) / n) whatever v is: the index is
    the first i with RN((i + 1) / n) > u0 -- O(1) instead of three n-element
    float64 arrays.  float64 weights: p[i] = RN(1/n) and the float64 cumsum
    rounds, so numpy's arithmetic is replayed (host bookkeeping of the random
    stream, O(n))."""
    if np.dtype(weight_dtype) == np.float64:
        w = np.ones(n, dtype=np.float64)
        p = w / w.sum()
        cdf = p.cumsum()
        cdf /= cdf[-1]
        return int(cdf.searchsorted(u0, side="right"))
    if n >= 2 ** 29:
        w = np.ones(n, dtype=np.float32)
        p = (w / w.sum()).astype(np.float64)
        cdf = p.cumsum()
        cdf /= cdf[-1]
        return int(cdf.searchsorted(u0, side="right"))
    i = max(0, int(u0 * n) - 2)
    while i < n and (i + 1) / n <= u0:     # Python float division rounds correctly
        i += 1
    return min(i, n - 1)


def _draws(rs: np.random.RandomState, k: int, L: int):
    """The random numbers _kmeans_plusplus consumes (sklearn/cluster/_kmeans.py:215-248):
    the first centre's random_sample() and, per later centre, uniform(size=L) --
    as their 53-bit mantissas.  One draw of (k - 1) * L doubles is the same stream
    in the same order (round 5: the per-centre Python loop cost ~4 ms per call
    at k = 1024; tests/test_kpp.py checks the equality)."""
    u0 = rs.random_sample()
    umant = np.zeros(max(1, (k - 1) * L), np.uint64)
    if k > 1:
        u = rs.uniform(size=(k - 1) * L)
        m = np.ldexp(u, 53)
        assert np.array_equal(np.ldexp(m, -53), u)      # random_sample doubles are multiples of 2**-53
        umant[:] = m.astype(np.uint64)
    return u0, umant


def kmeans_plusplus(X: torch.Tensor, n_clusters: int, *, random_state=None, n_local_trials=None,
                    weight_dtype=None):
    """GPU k-means++ of a (n, d) cloud on a HIP device; returns (centers (k, d) float32, indices int64).
    ``weight_dtype``: dtype of sklearn's unit sample weights for the first draw (X's dtype by default;
    the estimator passes float64 when it casts float64 points to float32)."""
    if not (isinstance(X, torch.Tensor) and X.is_cuda):
        raise _lib.PcmError("kmeans_plusplus expects a HIP device tensor (no CPU fallback)")
    if X.dim() != 2 or not 1 <= X.shape[1] <= 4:
        raise ValueError("X must be (n, d) with 1 <= d <= 4")
    Xf = X.to(torch.float32).contiguous()
    n, d = Xf.shape
    k = int(n_clusters)
    if not 1 <= k <= n:
        raise ValueError(f"n_samples={n} should be >= n_clusters={k}")
    rs = random_state if isinstance(random_state, np.random.RandomState) else np.random.RandomState(random_state)
    L = 2 + int(np.log(k)) if n_local_trials is None else int(n_local_trials)
    u0, umant = _draws(rs, k, L)
    if weight_dtype is None:
        weight_dtype = np.float64 if X.dtype == torch.float64 else np.float32
    first = _first_index(n, u0, weight_dtype)
    idx = torch.empty(k, dtype=torch.int64, device=Xf.device)
    lib = _lib.load()
    nbytes = ctypes.c_size_t()
    _lib.check(lib.pcm_kmeanspp_workspace(n, d, k, L, ctypes.byref(nbytes)), "pcm_kmeanspp_workspace")
    # device workspace from torch's caching allocator (reused by later calls)
    ws = torch.empty(int(nbytes.value), dtype=torch.uint8, device=Xf.device)
    rc = lib.pcm_kmeanspp(_ptr(Xf), n, d, k, L, first, umant.ctypes.data_as(ctypes.c_void_p), _ptr(idx), _ptr(ws),
                          nbytes.value, _stream())
    if rc == -4:
        raise ValueError("input points contain NaN or Inf")
    _lib.check(rc, "pcm_kmeanspp")
    return Xf[idx].clone(), idx
