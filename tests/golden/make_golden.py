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
  plugin/plugin_cloud_k{64,16}.npz  the cloud shape the plugin emits
                     (plugin.py:147-192): 65,917 points, pixel-unit y in
                     [0, 1500), x in [0, 2200), z = relative height shifted so
                     its 2nd percentile is 0 (negative below), float32 at the
                     boundary; k-means++ init (random_state 0 / 1); sklearn's
                     float64 Lloyd (the reference's dtype, plugin.py:192): a
                     tol=0 fit, a tol=1e-4 fit (_tolerance) and 5 steps; plus
                     the float32 sklearn fit.
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
    plugin_cloud()


def plugin_cloud():
    """Pixel-unit height-map cloud as plugin.py:147-192 emits it (restated by
    tests/fake_pipeline.pair_cloud): sparse valid pixels of a 1500 x 2200
    disparity map.  The reference's points are float64 (plugin.py:192) and
    scikit-learn keeps the input dtype, so the reference CPU path on this cloud
    is the float64 Lloyd on the (float32-cast) points; the float32 sklearn fit
    of the same points is recorded too (its GEMM-form rounding at pixel scale
    takes another trajectory: see DESIGN.md §2)."""
    import sys
    sys.path.insert(0, os.path.dirname(OUT))
    from fake_pipeline import pair_cloud
    from sklearn.cluster import kmeans_plusplus
    from sklearn.cluster._kmeans import _tolerance
    H, W = 1500, 2200
    rng = np.random.default_rng(7)
    yy, xx = np.mgrid[0:H, 0:W]
    disparity = -16.0 * (8 * np.sin(xx / 230.0) + 5 * np.cos(yy / 170.0) + 0.002 * xx + rng.normal(0, 0.3, (H, W)))
    height_map = -disparity / 16.0
    valid = rng.random((H, W)) < 0.02
    pts, _ = pair_cloud(height_map, valid)
    X = pts.astype(np.float32)                     # the GPU boundary cast
    X64 = X.astype(np.float64)
    for K, seed in ((64, 0), (16, 1)):
        C0 = kmeans_plusplus(X64, K, random_state=seed)[0].astype(np.float32)
        w64 = np.ones(X.shape[0])
        d = dict(X=X, C0=C0)
        lab, ine, cen, it = _kmeans_single_lloyd(X64, w64, C0.astype(np.float64), max_iter=300, tol=0.0, n_threads=1)
        d.update(f64_labels=lab, f64_centers=cen, f64_inertia=np.float64(ine), f64_n_iter=np.int64(it))
        tol = _tolerance(X64, 1e-4)
        lab, ine, cen, it = _kmeans_single_lloyd(X64, w64, C0.astype(np.float64), max_iter=300, tol=tol, n_threads=1)
        d.update(tol_abs=np.float64(tol), tol_labels=lab, tol_centers=cen, tol_inertia=np.float64(ine),
                 tol_n_iter=np.int64(it))
        lab, ine, cen, it = _kmeans_single_lloyd(X, np.ones(X.shape[0], np.float32), C0.copy(), max_iter=300,
                                                 tol=0.0, n_threads=1)
        d.update(f32_labels=lab, f32_centers=cen, f32_inertia=np.float64(ine), f32_n_iter=np.int64(it))
        # float64 steps from C0 (E-step labels, counts, new centres) via lloyd_iter_chunked_dense
        C = C0.astype(np.float64)
        rec = dict(step_c_in=[], step_labels=[], step_c_out=[], step_weight=[])
        for _ in range(5):
            Cn = np.zeros_like(C)
            wic = np.zeros(K)
            lb = np.full(X.shape[0], -1, dtype=np.int32)
            lloyd_iter_chunked_dense(X64, w64, C, Cn, wic, lb, np.zeros(K), 1)
            rec["step_c_in"].append(C.copy())
            rec["step_labels"].append(lb)
            rec["step_c_out"].append(Cn.copy())
            rec["step_weight"].append(wic.copy())
            C = Cn
        d.update({k_: np.stack(v) for k_, v in rec.items()})
        name = f"plugin_cloud_k{K}.npz"
        np.savez_compressed(os.path.join(OUT, "plugin", name), **d)
        print(name, {k: v.shape for k, v in d.items()})


if __name__ == "__main__":
    main()
