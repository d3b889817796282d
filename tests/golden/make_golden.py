"""Generate scikit-learn golden vectors for the Lloyd oracle (build container only).

The reference's only executed K-means is scikit-learn's Lloyd
(members/jasraj/land_use_classification/core.py:227-228 -> sklearn/cluster/
_kmeans.py:623 _kmeans_single_lloyd -> _k_means_lloyd.pyx:23 lloyd_iter_chunked_dense).
scikit-learn 1.7.2 is importable in the build container but is NOT available to
the tests at run time on the GPU box, so its outputs are frozen here as small
.npz fixtures (inputs + per-iteration outputs).  Re-run with:

    python tests/golden/make_golden.py

Fixtures (all float32, unit weights, n_threads=1):
  cfg1_n10k_k8.npz   SURVEY config 1 shape: N=10,000 K=8 D=3, init X[:8],
                     20 stepwise lloyd_iter_chunked_dense calls + full fit.
  n4096_k64.npz      N=4096 K=64 D=3, init X[sorted choice], 10 steps + fit.
  d4_fp16.npz        N=4096 K=16 D=4 (fp16 data widened to fp32), 6 steps.
  d2_k5.npz          N=2000 K=5 D=2, 8 steps.
  ties_dups.npz      duplicated points and duplicated centres (exact ties).
  empty_reloc.npz    an init that empties a cluster (one relocation).
  jasraj_obia_k5.npz the reference's only executed K-means call site
                     (members/jasraj/land_use_classification/core.py:225-228):
                     StandardScaler(X) of 1500 x 20 float64 superpixel-like
                     features, KMeans(n_clusters=5, random_state=42,
                     n_init=10).fit -> labels, centres, inertia, n_iter; plus
                     one _kmeans_single_lloyd run from X[:5] (float64) and the
                     kmeans_plusplus indices of random_state=42.
  dense_d8_f32.npz   600 x 8 float32, K=6: _kmeans_single_lloyd from X[:6].
"""
import os

import numpy as np
from sklearn.cluster._k_means_lloyd import lloyd_iter_chunked_dense
from sklearn.cluster._kmeans import _kmeans_single_lloyd

OUT = os.path.dirname(os.path.abspath(__file__))
OUT_DENSE = os.path.join(OUT, "dense")   # dense-path fixtures (other keys than the Lloyd step fixtures)


def steps(X, C0, n_steps):
    n, d = X.shape
    k = C0.shape[0]
    w = np.ones(n, dtype=X.dtype)
    C = C0.copy()
    rec = dict(c_in=[], labels=[], c_out=[], weight=[], shift=[])
    for _ in range(n_steps):
        Cn = np.zeros_like(C)
        wic = np.zeros(k, dtype=X.dtype)
        lab = np.full(n, -1, dtype=np.int32)
        sh = np.zeros(k, dtype=X.dtype)
        lloyd_iter_chunked_dense(X, w, C, Cn, wic, lab, sh, 1)
        rec["c_in"].append(C.copy())
        rec["labels"].append(lab.copy())
        rec["c_out"].append(Cn.copy())
        rec["weight"].append(wic.copy())
        rec["shift"].append(sh.copy())
        C = Cn
    return {k_: np.stack(v) for k_, v in rec.items()}


def fit(X, C0, max_iter=300):
    w = np.ones(X.shape[0], dtype=X.dtype)
    labels, inertia, centers, n_iter = _kmeans_single_lloyd(
        X, w, C0.copy(), max_iter=max_iter, tol=0.0, n_threads=1)
    return dict(fit_labels=labels, fit_inertia=np.float64(inertia), fit_centers=centers,
                fit_n_iter=np.int64(n_iter))


def save(name, X, C0, n_steps, do_fit=True, max_iter=300):
    d = dict(X=X, C0=C0)
    d.update(steps(X, C0, n_steps))
    if do_fit:
        d.update(fit(X, C0, max_iter))
    np.savez_compressed(os.path.join(OUT, name), **d)
    print(name, {k: v.shape for k, v in d.items()})


def main():
    X = np.random.default_rng(0).random((10_000, 3), dtype=np.float32)
    save("cfg1_n10k_k8.npz", X, X[:8].copy(), 20)

    X = np.random.default_rng(2).random((4096, 3), dtype=np.float32)
    idx = np.sort(np.random.default_rng(1).choice(4096, 64, replace=False))
    save("n4096_k64.npz", X, X[idx].copy(), 10)

    X = np.random.default_rng(3).random((4096, 4)).astype(np.float16).astype(np.float32)
    save("d4_fp16.npz", X, X[:16].copy(), 6)

    X = (np.random.default_rng(4).standard_normal((2000, 2)) * 50.0 + 300.0).astype(np.float32)
    save("d2_k5.npz", X, X[:5].copy(), 8)

    # exact ties: every point duplicated, two identical centres
    base = np.random.default_rng(5).integers(0, 8, size=(300, 3)).astype(np.float32)
    X = np.concatenate([base, base])
    C0 = np.stack([X[0], X[0], X[1], X[2], X[3]]).astype(np.float32)
    save("ties_dups.npz", X, C0, 4, do_fit=False)

    # a far initial centre receives no point -> relocation on the first step
    X = np.random.default_rng(6).random((500, 3), dtype=np.float32)
    C0 = np.concatenate([X[:3], np.array([[40.0, 40.0, 40.0]], dtype=np.float32)])
    save("empty_reloc.npz", X, C0, 3)

    jasraj()
    dense_f32()


def obia_features(n=1500, d=20, seed=42):
    """Superpixel-feature-like rows (LAB means/stds, Gabor energies, entropy:
    mixed scales and correlated groups), 7 land-cover classes."""
    rng = np.random.default_rng(seed)
    proto = rng.normal(0, 1, (7, d)) * rng.uniform(0.5, 3.0, d) + rng.uniform(-5, 50, d)
    cls = rng.integers(0, 7, n)
    X = proto[cls] + rng.normal(0, 1, (n, d)) * rng.uniform(0.3, 2.0, d)
    X[:, 3:6] = np.abs(X[:, 3:6])                     # std-like features
    X[:, -1] = np.log1p(np.abs(X[:, -1]))             # entropy-like
    return X.astype(np.float64)


def jasraj():
    from sklearn.cluster import KMeans, kmeans_plusplus
    from sklearn.preprocessing import StandardScaler
    Xs = StandardScaler().fit_transform(obia_features())          # core.py:225-226
    km = KMeans(n_clusters=5, random_state=42, n_init=10).fit(Xs)  # core.py:227-228
    w = np.ones(Xs.shape[0])
    lab1, in1, cen1, it1 = _kmeans_single_lloyd(Xs, w, Xs[:5].copy(), max_iter=300, tol=0.0, n_threads=1)
    _, kidx = kmeans_plusplus(Xs, 5, random_state=42)
    d = dict(X=Xs, labels=km.labels_.astype(np.int32), centers=km.cluster_centers_, inertia=np.float64(km.inertia_),
             n_iter=np.int64(km.n_iter_), single_labels=lab1, single_centers=cen1, single_inertia=np.float64(in1),
             single_n_iter=np.int64(it1), kpp_indices=kidx.astype(np.int64))
    np.savez_compressed(os.path.join(OUT_DENSE, "jasraj_obia_k5.npz"), **d)
    print("jasraj_obia_k5.npz", {k: v.shape for k, v in d.items()})


def dense_f32():
    X = obia_features(600, 8, seed=3).astype(np.float32)
    w = np.ones(X.shape[0], dtype=np.float32)
    lab, ine, cen, it = _kmeans_single_lloyd(X, w, X[:6].copy(), max_iter=300, tol=0.0, n_threads=1)
    d = dict(X=X, C0=X[:6].copy(), fit_labels=lab, fit_centers=cen, fit_inertia=np.float64(ine), fit_n_iter=np.int64(it))
    np.savez_compressed(os.path.join(OUT_DENSE, "dense_d8_f32.npz"), **d)
    print("dense_d8_f32.npz", {k: v.shape for k, v in d.items()})


if __name__ == "__main__":
    main()
