"""Generic-D (dense) Lloyd K-means and k-means++ on the GPU.

The reference's only executed K-means is
``KMeans(n_clusters=5, random_state=42, n_init=10).fit_predict(StandardScaler(X))``
on ~1500 x 20 float64 superpixel features
(``members/jasraj/land_use_classification/core.py:225-228``).  Point clouds
(D <= 4, float32) go through the pruned engine (``engine.py``); feature
vectors go through ``csrc/pcm_dense.hip``: brute force over all K with the
centres in LDS, computed in the input precision (float64 stays float64, as in
scikit-learn), exact integer sums, everything on the device.  There is no CPU
fallback.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from .engine import _ptr, _stream
from .fixed import inertia_from_limbs

PCM_F32, PCM_F64 = 0, 2
DMAX = 64


def _dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float64:
        return PCM_F64
    if t.dtype == torch.float32:
        return PCM_F32
    raise ValueError("dense path: points must be float32 or float64")


@dataclass
class DenseResult:
    labels: torch.Tensor
    centers: torch.Tensor
    inertia: float
    n_iter: int
    strict: bool
    changed: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int64))
    shift: np.ndarray = field(default_factory=lambda: np.zeros(0))
    relocations: int = 0


def _check(X: torch.Tensor):
    if not (isinstance(X, torch.Tensor) and X.is_cuda):
        raise _lib.PcmError("dense path expects a HIP device tensor (no CPU fallback)")
    if X.dim() != 2 or not 1 <= X.shape[1] <= DMAX:
        raise ValueError(f"X must be (n, d) with 1 <= d <= {DMAX}")
    return X.contiguous()


def dense_fit(X: torch.Tensor, centers_init: torch.Tensor, max_iter: int = 300, tol: float = 0.0,
              chunk: int = 8) -> DenseResult:
    """One ``_kmeans_single_lloyd`` run (sklearn/cluster/_kmeans.py:623-752) on (n, d) rows
    in X's precision; ``tol`` is absolute (sklearn's ``_tolerance`` output)."""
    X = _check(X)
    n, d = X.shape
    C0 = centers_init.to(device=X.device, dtype=X.dtype).contiguous()
    k = C0.shape[0]
    if C0.shape[1] != d or not 1 <= k <= n:
        raise ValueError("centers_init must be (k, d) with 1 <= k <= n")
    if not torch.isfinite(X).all():
        raise ValueError("input points contain NaN or Inf")
    lib = _lib.load()
    h = ctypes.c_void_p()
    _lib.check(lib.pcm_dense_create(X.device.index, n, d, k, _dtype_code(X), int(max_iter), ctypes.byref(h)),
               "pcm_dense_create")
    try:
        maxabs = np.ascontiguousarray(X.abs().amax(0).double().cpu().numpy())
        _lib.check(lib.pcm_dense_begin(h, _ptr(X), maxabs.ctypes.data_as(ctypes.c_void_p), _ptr(C0), float(tol),
                                       int(max_iter), _stream()), "pcm_dense_begin")
        st = _lib.PcmStatus()
        it = 0
        while True:
            _lib.check(lib.pcm_dense_iterate(h, max(1, min(chunk, max_iter - it)), _stream()), "pcm_dense_iterate")
            _lib.check(lib.pcm_dense_status(h, ctypes.byref(st), _stream()), "pcm_dense_status")
            it = int(st.iter)
            if st.done:
                break
        _lib.check(lib.pcm_dense_final(h, _stream()), "pcm_dense_final")
        _lib.check(lib.pcm_dense_status(h, ctypes.byref(st), _stream()), "pcm_dense_status")
        labels = torch.empty(n, dtype=torch.int32, device=X.device)
        centers = torch.empty((k, d), dtype=X.dtype, device=X.device)
        ch = np.zeros(max_iter, np.uint64)
        sh = np.zeros(max_iter, np.float64)
        _lib.check(lib.pcm_dense_outputs(h, _ptr(labels), _ptr(centers), ch.ctypes.data_as(ctypes.c_void_p),
                                         sh.ctypes.data_as(ctypes.c_void_p), int(max_iter), _stream()),
                   "pcm_dense_outputs")
        inertia = inertia_from_limbs(list(st.inertia_limbs), st.inertia_scale, st.inertia_overflow)
        return DenseResult(labels=labels, centers=centers, inertia=inertia, n_iter=it, strict=st.done == 1,
                           changed=ch[:it].astype(np.int64), shift=sh[:it], relocations=int(st.list_rebuilds))
    finally:
        lib.pcm_dense_destroy(h)


def _kpp_scale(n: int, maxd: float) -> int:
    if maxd <= 0 or n <= 0:
        return 0
    _, e = math.frexp(maxd * (1.0 + 2.0 ** -20))
    return int(62 - max(1, int(n - 1).bit_length()) - e)


def dense_kmeanspp(X: torch.Tensor, n_clusters: int, *, random_state=None, n_local_trials=None):
    """k-means++ (sklearn/cluster/_kmeans.py:174-272) in X's precision; returns (centers, indices)."""
    from .kpp import _first_index
    X = _check(X)
    n, d = X.shape
    k = int(n_clusters)
    if not 1 <= k <= n:
        raise ValueError(f"n_samples={n} should be >= n_clusters={k}")
    if not torch.isfinite(X).all():      # before any weight is formed (kmeans_plusplus raises likewise)
        raise ValueError("input points contain NaN or Inf")
    rs = random_state if isinstance(random_state, np.random.RandomState) else np.random.RandomState(random_state)
    L = 2 + int(np.log(k)) if n_local_trials is None else int(n_local_trials)
    u0 = rs.random_sample()
    umant = np.zeros(max(1, (k - 1) * L), np.uint64)
    for c in range(1, k):
        u = rs.uniform(size=L)
        umant[(c - 1) * L:c * L] = np.ldexp(u, 53).astype(np.uint64)
    ext = (X.amax(0).double() - X.amin(0).double()).cpu().numpy()
    s = _kpp_scale(n, float((ext * ext).sum()))
    idx = torch.empty(k, dtype=torch.int64, device=X.device)
    lib = _lib.load()
    nbytes = ctypes.c_size_t()
    _lib.check(lib.pcm_dense_kmeanspp_workspace(n, d, _dtype_code(X), k, L, ctypes.byref(nbytes)),
               "pcm_dense_kmeanspp_workspace")
    ws = torch.empty(int(nbytes.value), dtype=torch.uint8, device=X.device)
    # sklearn's unit sample weights are in X's dtype: the first draw follows numpy's choice() for it
    first = _first_index(n, u0, np.float64 if X.dtype == torch.float64 else np.float32)
    _lib.check(lib.pcm_dense_kmeanspp(_ptr(X), n, d, _dtype_code(X), k, L, first,
                                      umant.ctypes.data_as(ctypes.c_void_p), s, _ptr(idx), _ptr(ws), nbytes.value,
                                      _stream()), "pcm_dense_kmeanspp")
    return X[idx].clone(), idx
