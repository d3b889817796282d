"""``KMeans`` estimator: the reference's only K-means call site on the GPU engine.

The reference runs ``KMeans(n_clusters=K, random_state=42, n_init=10).fit_predict(X)``
(``members/jasraj/land_use_classification/core.py:227-228``).
This class keeps that API and restates the control flow of scikit-learn 1.7.2's
``KMeans.fit`` (``sklearn/cluster/_kmeans.py:1427-1547``):

* ``tol`` becomes ``mean(var(X, axis=0)) * tol`` (``_tolerance``, ``:279-287``),
  computed on the input exactly as sklearn does (NumPy, the input dtype);
* X is centred by its mean before fitting and the mean is added back to the
  centres (``:1479-1484``, ``:1536-1537``);
* ``n_init`` runs share ONE ``RandomState``; each is seeded by k-means++
  (``_kmeans_plusplus``), ``'random'`` rows or a given array (``_init_centroids``,
  ``:955-1032``); a run replaces the best only if its inertia is lower and its
  clustering differs (``_is_same_clustering``, ``_k_means_common.pyx:314-328``);
  ``n_init='auto'`` is 1 for k-means++ / an array, 10 for ``'random'``.

Every pass over the data runs in the HIP kernels (k-means++ seeding, Lloyd
iterations, final E-step); the host holds only O(K) state plus the mean/var of
the boundary, which mirror sklearn's own NumPy calls.  Dtypes follow sklearn
(float32 stays float32, everything else becomes float64):

* float32 point clouds (D <= 4): the pruned point-cloud engine (``lloyd_fit``,
  ``kmeans_plusplus``; canonical float32 arithmetic);
* D > 4, or float64 input the dense engine can take (the reference's
  1500 x 20 float64 call site): the dense engine (``dense.py``), computing in the
  input precision;
* float64 point clouds (D <= 4) stay float64 on the dense engine whatever
  their size (as scikit-learn keeps float64).  ``float64_points="float32"`` opts
  in to casting large ones -- centres beyond the dense engine's 64 KB LDS stage
  (K * D * 8 bytes) or more than 2**26 distance evaluations per iteration
  (N * K) -- to float32 for the pruned engine (the boundary cast of the plugin
  path: its canonical fp32 fit equals sklearn's float64 fit on pixel-unit
  height-map clouds, tests/test_plugin_cloud_golden.py; on general float64 data
  labels may differ from sklearn's float64 fit, so the cast warns).  The
  k-means++ first draw then still uses float64 unit weights, as sklearn's.
"""
from __future__ import annotations

from typing import Callable, Optional

import warnings

import numpy as np


def _same_clustering(l1: np.ndarray, l2: np.ndarray, k: int) -> bool:
    """sklearn ``_is_same_clustering``: labels1 -> labels2 is a consistent mapping."""
    mapping = np.full(k, -1, dtype=np.int64)
    _, first = np.unique(l1, return_index=True)
    mapping[l1[first]] = l2[first]
    return bool(np.array_equal(mapping[l1], l2))


class KMeans:
    """Drop-in for ``sklearn.cluster.KMeans`` (Lloyd, dense, unit weights) on MI355X."""

    def __init__(self, n_clusters: int = 8, *, init="k-means++", n_init="auto", max_iter: int = 300,
                 tol: float = 1e-4, random_state=None, algorithm: str = "lloyd", float64_points: str = "dense",
                 _fit: Optional[Callable] = None, _seed: Optional[Callable] = None):
        if float64_points not in ("dense", "float32"):
            raise ValueError("float64_points must be 'dense' or 'float32'")
        self.n_clusters = n_clusters
        self.init = init
        self.n_init = n_init
        self.max_iter = max_iter
        self.tol = tol
        self.random_state = random_state
        self.algorithm = algorithm
        self.float64_points = float64_points
        self._fit = _fit      # tests: a CPU stand-in for (Xc, C0, max_iter, tol) -> (labels, centers, inertia, n_iter)
        self._seed = _seed    # tests: a CPU stand-in for k-means++ (Xc, k, RandomState) -> centers

    # ------------------------------------------------------------ GPU legs
    DENSE_LDS_BYTES = 64 * 1024        # the dense engine stages all K centres in LDS (pcm_dense.hip)
    DENSE_MAX_EVALS = 1 << 26          # N * K distance evaluations per brute-force iteration

    @staticmethod
    def _dense(X: np.ndarray, k: int, float64_points: str = "dense") -> bool:
        """Which engine fits X with k clusters: True = dense (input precision), False = pruned (float32)."""
        n, d = X.shape
        if d > 4:
            return True
        if X.dtype != np.float64:
            return False
        if float64_points == "dense":
            return True
        return k * d * 8 <= KMeans.DENSE_LDS_BYTES and n * k <= KMeans.DENSE_MAX_EVALS

    def _gpu_fit(self, Xc: np.ndarray, C0: np.ndarray, max_iter: int, tol: float):
        import torch

        if KMeans._dense(Xc, C0.shape[0], self.float64_points):
            from .dense import dense_fit
            res = dense_fit(torch.from_numpy(Xc).cuda(), torch.from_numpy(np.ascontiguousarray(C0, Xc.dtype)).cuda(),
                            max_iter=max_iter, tol=tol)
        else:
            from .lloyd import LOCAL, lloyd_fit
            Xf = np.ascontiguousarray(Xc, np.float32)
            res = lloyd_fit(torch.from_numpy(Xf).cuda(), torch.from_numpy(np.ascontiguousarray(C0, np.float32)).cuda(),
                            max_iter=max_iter, tol=tol, group=LOCAL)
        torch.cuda.synchronize()
        return res.labels.cpu().numpy(), res.centers.cpu().numpy(), float(res.inertia), int(res.n_iter)

    def _gpu_seed(self, Xc: np.ndarray, k: int, rs: np.random.RandomState) -> np.ndarray:
        import torch

        if KMeans._dense(Xc, k, self.float64_points):
            from .dense import dense_kmeanspp
            C, _ = dense_kmeanspp(torch.from_numpy(Xc).cuda(), k, random_state=rs)
        else:
            from .kpp import kmeans_plusplus
            # sklearn's unit sample weights are in X's dtype: the first draw keeps them float64
            C, _ = kmeans_plusplus(torch.from_numpy(np.ascontiguousarray(Xc, np.float32)).cuda(), k, random_state=rs,
                                   weight_dtype=Xc.dtype)
        return C.cpu().numpy().astype(Xc.dtype)

    # ------------------------------------------------------------ sklearn API
    def fit(self, X, y=None, sample_weight=None):
        if sample_weight is not None and not np.all(np.asarray(sample_weight) == 1):
            raise NotImplementedError("unit sample weights only (the reference's call site passes none)")
        if self.algorithm != "lloyd":
            raise NotImplementedError("algorithm='lloyd' only")
        if hasattr(X, "detach"):
            X = X.detach().cpu().numpy()
        X = np.asarray(X)
        dt = np.float32 if X.dtype == np.float32 else np.float64     # sklearn: dtype=[float64, float32]
        X = np.array(X, dtype=dt, order="C", copy=True)
        if X.ndim != 2:
            raise ValueError("Expected a 2D array")
        if not np.isfinite(X).all():                                      # sklearn check_array
            raise ValueError("Input X contains NaN or infinity.")
        n, d = X.shape
        k = int(self.n_clusters)
        if self._fit is None and dt == np.float64 and not KMeans._dense(X, k, self.float64_points):
            warnings.warn("pcm_amd.KMeans: float64 points cast to float32 for the pruned engine (float64_points="
                          "'float32'); labels may differ from a float64 fit", RuntimeWarning, stacklevel=2)
        if n < k:
            raise ValueError(f"n_samples={n} should be >= n_clusters={k}.")
        init = self.init
        init_is_array = not isinstance(init, str)
        if self.n_init == "auto":
            n_init = 10 if (isinstance(init, str) and init == "random") else 1
        else:
            n_init = int(self.n_init)
        if init_is_array and n_init != 1:
            n_init = 1    # sklearn warns and runs once for an explicit init array
        if isinstance(self.random_state, np.random.RandomState):
            rs = self.random_state
        elif self.random_state is None:          # sklearn check_random_state(None): numpy's global RandomState
            rs = np.random.mtrand._rand
        else:
            rs = np.random.RandomState(self.random_state)
        tol_abs = float(np.mean(np.var(X, axis=0)) * self.tol) if self.tol else 0.0   # _tolerance (X's dtype)
        X_mean = X.mean(axis=0)
        Xc = X - X_mean                                                              # centring (:1479-1484)
        fit = self._fit or self._gpu_fit
        seed = self._seed or self._gpu_seed
        best = None
        for _ in range(n_init):
            if init_is_array:
                C0 = np.asarray(init, dtype=dt) - X_mean
            elif init == "k-means++":
                C0 = seed(Xc, k, rs)
            elif init == "random":
                sw = np.ones(n, dtype=X.dtype)                               # _check_sample_weight
                C0 = Xc[rs.choice(n, size=k, replace=False, p=sw / sw.sum())]
            else:
                raise ValueError(f"init must be 'k-means++', 'random' or an array, got {init!r}")
            labels, centers, inertia, n_iter = fit(Xc, C0, int(self.max_iter), tol_abs)
            if best is None or (inertia < best[2] and not _same_clustering(labels, best[0], k)):
                best = (labels, centers, inertia, n_iter)
        labels, centers, inertia, n_iter = best
        self.cluster_centers_ = (centers + X_mean).astype(dt)
        self.labels_ = labels.astype(np.int32)
        self.inertia_ = dt(inertia)           # sklearn returns the inertia in X's dtype
        self.n_iter_ = n_iter
        self.n_features_in_ = d
        return self

    def fit_predict(self, X, y=None, sample_weight=None):
        return self.fit(X, sample_weight=sample_weight).labels_
