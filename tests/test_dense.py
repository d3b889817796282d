"""Dense (generic-D) path, SURVEY.md §8 row a9: the reference's only executed
K-means call site, ``KMeans(n_clusters=5, random_state=42, n_init=10).fit_predict(
StandardScaler(X))`` on ~1500 x 20 float64 features
(members/jasraj/land_use_classification/core.py:225-228).

CPU: the dense oracle (oracle/dense_ref.py) and the float64 k-means++ oracle
are pinned to scikit-learn golden runs (tests/golden/dense/*.npz, generated in
the build container by tests/golden/make_golden.py); the estimator driven by
the oracle legs reproduces scikit-learn's KMeans on the call-site fixture.
GPU: the HIP dense engine (csrc/pcm_dense.hip, through the C ABI) equals the
oracle bit for bit and scikit-learn's labels / n_iter on the fixture.
"""
import os

import numpy as np
import pytest

from oracle import dense_ref as DR
from oracle import kpp_ref as P

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "dense")


def jasraj():
    return np.load(os.path.join(GOLD, "jasraj_obia_k5.npz"))


def oracle_fit(Xc, C0, max_iter, tol):
    r = DR.dense_fit(Xc, C0, max_iter=max_iter, tol=tol)
    return r["labels"], r["centers"], r["inertia"], r["n_iter"]


def oracle_seed(Xc, k, rs):
    return P.kmeanspp(Xc, k, rs, keep_dtype=True)[0]


def test_dense_oracle_matches_sklearn_single_run():
    g = jasraj()
    X = g["X"]
    r = DR.dense_fit(X, X[:5], max_iter=300, tol=0.0)
    np.testing.assert_array_equal(r["labels"], g["single_labels"])
    assert r["n_iter"] == int(g["single_n_iter"])
    np.testing.assert_allclose(r["centers"], g["single_centers"], rtol=1e-12, atol=1e-12)
    assert r["inertia"] == pytest.approx(float(g["single_inertia"]), rel=1e-12)


def test_dense_oracle_float32_d8():
    g = np.load(os.path.join(GOLD, "dense_d8_f32.npz"))
    r = DR.dense_fit(g["X"], g["C0"], max_iter=300, tol=0.0)
    assert r["centers"].dtype == np.float32
    np.testing.assert_array_equal(r["labels"], g["fit_labels"])
    assert r["n_iter"] == int(g["fit_n_iter"])
    np.testing.assert_allclose(r["centers"], g["fit_centers"], rtol=1e-5, atol=1e-5)
    assert r["inertia"] == pytest.approx(float(g["fit_inertia"]), rel=1e-5)


def test_float64_kmeanspp_oracle_matches_sklearn():
    g = jasraj()
    _, idx = P.kmeanspp(g["X"], 5, 42, keep_dtype=True)
    np.testing.assert_array_equal(idx, g["kpp_indices"])


def test_estimator_oracle_legs_reproduce_call_site():
    """KMeans(n_clusters=5, random_state=42, n_init=10).fit_predict on the
    StandardScaled 1500 x 20 float64 fixture: labels, n_iter, centres."""
    import pcm_amd
    g = jasraj()
    est = pcm_amd.KMeans(n_clusters=5, random_state=42, n_init=10, _fit=oracle_fit, _seed=oracle_seed)
    labels = est.fit_predict(g["X"])
    np.testing.assert_array_equal(labels, g["labels"])
    assert est.n_iter_ == int(g["n_iter"])
    assert est.cluster_centers_.dtype == np.float64 and isinstance(est.inertia_, np.float64)
    np.testing.assert_allclose(est.cluster_centers_, g["centers"], rtol=1e-10, atol=1e-10)
    assert est.inertia_ == pytest.approx(float(g["inertia"]), rel=1e-10)


def test_estimator_random_state_none_uses_global_stream():
    """random_state=None draws from numpy's global RandomState, as sklearn's
    check_random_state(None) does: np.random.seed(...) makes it repeatable."""
    import pcm_amd
    g = jasraj()
    out = []
    for _ in range(2):
        np.random.seed(123)
        est = pcm_amd.KMeans(n_clusters=5, n_init=2, _fit=oracle_fit, _seed=oracle_seed)
        out.append(est.fit_predict(g["X"][:400]))
    np.testing.assert_array_equal(out[0], out[1])


# ---------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pcm_amd
    return torch, pcm_amd


@pytest.mark.gpu
def test_gpu_dense_fit_matches_oracle_float64(gpu):
    torch, pcm = gpu
    from pcm_amd.dense import dense_fit
    g = jasraj()
    X = g["X"]
    ref = DR.dense_fit(X, X[:5], max_iter=300, tol=0.0)
    res = dense_fit(torch.from_numpy(X).cuda(), torch.from_numpy(X[:5].copy()).cuda(), max_iter=300, tol=0.0)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(res.labels.cpu().numpy(), ref["labels"])
    np.testing.assert_array_equal(res.centers.cpu().numpy(), ref["centers"])
    assert res.n_iter == ref["n_iter"]
    assert res.inertia == ref["inertia"]
    np.testing.assert_array_equal(res.shift, np.array(ref["shift"]))
    np.testing.assert_array_equal(res.labels.cpu().numpy(), g["single_labels"])   # and sklearn's


@pytest.mark.gpu
@pytest.mark.parametrize("n,d,k,dtype,tol", [(600, 8, 6, np.float32, 0.0), (5000, 33, 17, np.float64, 1e-6),
                                             (3000, 7, 40, np.float32, 0.0), (1, 5, 1, np.float64, 0.0),
                                             # centres past the 64 KB LDS stage: read from L2
                                             (6000, 6, 1500, np.float64, 0.0)])
def test_gpu_dense_fit_random(gpu, n, d, k, dtype, tol):
    torch, pcm = gpu
    from pcm_amd.dense import dense_fit
    rng = np.random.default_rng(n + d)
    X = (rng.normal(0, 1, (n, d)) * rng.uniform(0.1, 5, d)).astype(dtype)
    C0 = X[:k].copy()
    ref = DR.dense_fit(X, C0, max_iter=60, tol=tol)
    res = dense_fit(torch.from_numpy(X).cuda(), torch.from_numpy(C0).cuda(), max_iter=60, tol=tol)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(res.labels.cpu().numpy(), ref["labels"])
    np.testing.assert_array_equal(res.centers.cpu().numpy(), ref["centers"])
    assert res.n_iter == ref["n_iter"] and res.inertia == ref["inertia"]


@pytest.mark.gpu
def test_gpu_dense_relocation(gpu):
    torch, pcm = gpu
    from pcm_amd.dense import dense_fit
    rng = np.random.default_rng(5)
    X = rng.normal(0, 1, (2000, 12))
    C0 = np.concatenate([X[:4], np.full((3, 12), 40.0) + np.arange(3)[:, None]])   # 3 empty clusters
    ref = DR.dense_fit(X, C0, max_iter=40)
    res = dense_fit(torch.from_numpy(X).cuda(), torch.from_numpy(C0).cuda(), max_iter=40)
    torch.cuda.synchronize()
    assert res.relocations >= 1
    np.testing.assert_array_equal(res.labels.cpu().numpy(), ref["labels"])
    np.testing.assert_array_equal(res.centers.cpu().numpy(), ref["centers"])
    assert res.n_iter == ref["n_iter"]


@pytest.mark.gpu
def test_gpu_dense_kmeanspp(gpu):
    torch, pcm = gpu
    from pcm_amd.dense import dense_kmeanspp
    g = jasraj()
    _, idx = dense_kmeanspp(torch.from_numpy(g["X"]).cuda(), 5, random_state=42)
    np.testing.assert_array_equal(idx.cpu().numpy(), g["kpp_indices"])   # = sklearn.kmeans_plusplus
    X = np.random.default_rng(2).normal(0, 1, (20000, 24)).astype(np.float32)
    _, ir = P.kmeanspp(X, 50, 9, keep_dtype=True)
    _, ig = dense_kmeanspp(torch.from_numpy(X).cuda(), 50, random_state=9)
    np.testing.assert_array_equal(ig.cpu().numpy(), ir)


@pytest.mark.gpu
def test_gpu_estimator_call_site(gpu):
    """The call site itself on the GPU: pcm_amd.KMeans(n_clusters=5, random_state=42,
    n_init=10).fit_predict(1500 x 20 float64) == scikit-learn's labels."""
    torch, pcm = gpu
    g = jasraj()
    est = pcm.KMeans(n_clusters=5, random_state=42, n_init=10)
    labels = est.fit_predict(g["X"])
    np.testing.assert_array_equal(labels, g["labels"])
    assert est.n_iter_ == int(g["n_iter"])
    np.testing.assert_allclose(est.cluster_centers_, g["centers"], rtol=1e-10, atol=1e-10)
    ref = pcm.KMeans(n_clusters=5, random_state=42, n_init=10, _fit=oracle_fit, _seed=oracle_seed).fit(g["X"])
    np.testing.assert_array_equal(est.cluster_centers_, ref.cluster_centers_)
    assert est.inertia_ == ref.inertia_


# ---------------------------------------------------------------- ADVICE r2 (routing, first draw, NaN)
def test_first_index_matches_numpy_choice_float64_and_float32():
    """kpp._first_index replays RandomState.choice(n, p=w / w.sum()) for sklearn's unit
    weights in X's dtype (float64 weights: the rounded cumsum is replayed)."""
    from pcm_amd.kpp import _first_index
    for n in (1, 2, 3, 7, 1500, 4097, 100_003):
        for seed in range(12):
            for dt in (np.float32, np.float64):
                rs = np.random.RandomState(seed)
                w = np.ones(n, dtype=dt)
                want = rs.choice(n, p=w / w.sum())
                u0 = np.random.RandomState(seed).random_sample()
                assert _first_index(n, u0, dt) == want, (n, seed, dt)


def test_estimator_engine_routing():
    from pcm_amd.estimator import KMeans
    f64, f32 = np.zeros((1500, 20)), np.zeros((1500, 3), np.float32)
    assert KMeans._dense(f64, 5)                                    # the call site: dense, float64
    assert KMeans._dense(np.zeros((1000, 3)), 8)                    # small float64 cloud: dense
    assert not KMeans._dense(f32, 8)                                # float32 cloud: pruned engine
    assert KMeans._dense(np.zeros((1000, 3)), 4096)                 # float64 stays float64 (dense) by default
    assert KMeans._dense(np.zeros((200_000, 4)), 1024)
    assert not KMeans._dense(np.zeros((1000, 3)), 4096, "float32")  # opt-in cast: K*D*8 > 64 KB -> pruned
    assert not KMeans._dense(np.zeros((200_000, 4)), 1024, "float32")   # N*K > 2^26 -> pruned
    assert KMeans._dense(np.zeros((1000, 3)), 8, "float32")         # small float64 cloud: dense either way
    assert KMeans._dense(np.zeros((10, 5), np.float32), 3)          # D > 4: dense whatever the dtype
    with pytest.raises(ValueError):
        KMeans(4, float64_points="half")


def test_estimator_float32_cast_warns_and_keeps_float64_first_draw(monkeypatch):
    """The opt-in float32 cast warns, and the k-means++ first draw uses float64 unit weights."""
    from pcm_amd import estimator
    seen = {}

    def fake_seed(self, Xc, k, rs):
        seen["dtype"] = Xc.dtype
        return Xc[:k].copy()

    def fake_fit(self, Xc, C0, max_iter, tol):
        return np.zeros(len(Xc), np.int32), C0, 0.0, 1
    monkeypatch.setattr(estimator.KMeans, "_gpu_seed", fake_seed)
    monkeypatch.setattr(estimator.KMeans, "_gpu_fit", fake_fit)
    X = np.random.default_rng(0).random((70_000, 3))
    with pytest.warns(RuntimeWarning, match="float32"):
        estimator.KMeans(1024, float64_points="float32", n_init=1).fit(X)
    assert seen["dtype"] == np.float64


def test_estimator_rejects_nonfinite_before_any_device_call():
    from pcm_amd.estimator import KMeans

    def never(*a, **k):
        raise AssertionError("must not be reached")
    X = np.random.default_rng(0).random((100, 3))
    X[7, 1] = np.nan
    with pytest.raises(ValueError, match="NaN"):
        KMeans(4, _fit=never, _seed=never).fit(X)


@pytest.mark.gpu
def test_gpu_estimator_float64_cloud_large_k(gpu):
    """float64 D=3 cloud with K=4096 (beyond the dense engine's LDS stage) and the
    opt-in float32 cast: the estimator routes it to the pruned engine and fits;
    labels equal the oracle's canonical fit of the float32-cast centred cloud."""
    from pcm_amd.estimator import KMeans
    from oracle import lloyd_ref as R
    rng = np.random.default_rng(5)
    X = rng.random((60_000, 3)) * np.array([30.0, 1500.0, 2200.0])
    init = X[np.sort(rng.choice(len(X), 4096, replace=False))]
    with pytest.warns(RuntimeWarning):
        km = KMeans(4096, init=init, n_init=1, max_iter=15, tol=0.0, float64_points="float32").fit(X)
    Xc = X - X.mean(axis=0)
    ref = R.lloyd_fit(Xc.astype(np.float32), (init - X.mean(axis=0)).astype(np.float32), max_iter=15, tol=0.0,
                      fast=True)
    np.testing.assert_array_equal(km.labels_, ref["labels"])
    assert km.n_iter_ == ref["n_iter"] and km.cluster_centers_.dtype == np.float64


@pytest.mark.gpu
def test_gpu_estimator_float64_cloud_large_k_stays_float64(gpu):
    """Default routing: a float64 D=3 cloud with K*D*8 > 64 KB and
    N*K > 2^26 stays float64 on the dense engine; the fit equals the float64
    dense oracle on the centred cloud (labels, centres, n_iter)."""
    from pcm_amd.estimator import KMeans
    rng = np.random.default_rng(6)
    X = rng.random((40_000, 3)) * np.array([30.0, 1500.0, 2200.0])
    init = X[np.sort(rng.choice(len(X), 3000, replace=False))]
    km = KMeans(3000, init=init, n_init=1, max_iter=6, tol=0.0).fit(X)
    mu = X.mean(axis=0)
    ref = DR.dense_fit(X - mu, init - mu, max_iter=6, tol=0.0)
    np.testing.assert_array_equal(km.labels_, ref["labels"])
    np.testing.assert_array_equal(km.cluster_centers_, ref["centers"] + mu)
    assert km.n_iter_ == ref["n_iter"] and km.cluster_centers_.dtype == np.float64


@pytest.mark.gpu
def test_gpu_dense_kmeanspp_rejects_nan(gpu):
    import torch
    from pcm_amd.dense import dense_kmeanspp
    X = torch.rand(500, 6, dtype=torch.float64, device="cuda")
    X[3, 2] = float("nan")
    with pytest.raises(ValueError, match="NaN"):
        dense_kmeanspp(X, 4, random_state=0)
