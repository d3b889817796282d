"""CPU: pin the oracle (oracle/lloyd_ref.py + oracle/lloyd_ref.c) before trusting it.

1. scikit-learn golden vectors (tests/golden/*.npz, made by make_golden.py in
   the build container from sklearn 1.7.2 -- the Lloyd the reference executes,
   members/jasraj/land_use_classification/core.py:227-228):
   labels must be EXACT at every recorded step and for the full fit, n_iter
   equal; centres within 1e-5 relative (sklearn accumulates in float32,
   the oracle in exact fixed point).
2. scikit-learn's hand-computed known answers, restated as numbers
   (sklearn/cluster/tests/test_k_means.py:62-82, 85-112, 115-156).
3. numpy and C restatements agree bit for bit.
"""
import glob
import os

import numpy as np
import pytest

from oracle import cref
from oracle import lloyd_ref as R

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FILES = sorted(glob.glob(os.path.join(GOLDEN, "*.npz")))


def rel_close(a, b, scale, rtol=1e-5):
    np.testing.assert_allclose(a, b, rtol=rtol, atol=rtol * scale)


@pytest.mark.parametrize("path", FILES, ids=os.path.basename)
def test_steps_match_sklearn(path):
    g = np.load(path)
    X = g["X"]
    q = R.fixed_q(X)
    scale = float(np.abs(X).max())
    for t in range(g["labels"].shape[0]):
        C = g["c_in"][t]
        lab, sums, cnt, _ = R.local_stats(X, C, np.full(len(X), -1, np.int32), q)
        np.testing.assert_array_equal(lab, g["labels"][t], err_msg=f"step {t}")
        if (cnt == 0).any():
            m = int((cnt == 0).sum())
            R.relocate(sums, cnt, R.far_candidates(X, C, lab, 0, m), q)
        np.testing.assert_array_equal(cnt, g["weight"][t].astype(np.int64))
        rel_close(R.average(sums, cnt, q, C), g["c_out"][t], scale)


@pytest.mark.parametrize("path", [f for f in FILES if "ties" not in f], ids=os.path.basename)
def test_fit_matches_sklearn(path):
    g = np.load(path)
    X = g["X"]
    r = R.lloyd_fit(X, g["C0"], max_iter=300, tol=0.0, fast=True)
    np.testing.assert_array_equal(r["labels"], g["fit_labels"])
    assert r["n_iter"] == int(g["fit_n_iter"])
    rel_close(r["centers"], g["fit_centers"], float(np.abs(X).max()))
    assert r["inertia"] == pytest.approx(float(g["fit_inertia"]), rel=1e-5)


def test_known_answer_weighted_toy():
    """test_kmeans_results (test_k_means.py:62-82): weights [3,1,1,3]."""
    X = np.array([[0, 0], [0.5, 0], [0.5, 1], [1, 1]], dtype=np.float32)
    r = R.lloyd_fit(X, np.array([[0, 0], [1, 1]], np.float32), max_iter=300, weights=[3, 1, 1, 3])
    np.testing.assert_array_equal(r["labels"], [0, 0, 1, 1])
    np.testing.assert_allclose(r["centers"], [[0.125, 0], [0.875, 1]])
    assert r["inertia"] == pytest.approx(0.375)
    assert r["n_iter"] == 2


def test_known_answer_relocated_cluster():
    """test_kmeans_relocated_clusters (:85-112): the far centre is emptied and
    relocated; ties in distance go to the lowest point index -> the second of
    sklearn's two accepted outcomes."""
    X = np.array([[0, 0], [0.5, 0], [0.5, 1], [1, 1]], dtype=np.float32)
    r = R.lloyd_fit(X, np.array([[0.5, 0.5], [3, 3]], np.float32), max_iter=300)
    assert r["n_iter"] == 3
    assert r["inertia"] == pytest.approx(0.25)
    np.testing.assert_array_equal(r["labels"], [1, 1, 0, 0])
    np.testing.assert_allclose(r["centers"], [[0.75, 1.0], [0.25, 0.0]])


def test_known_answer_relocate_helper():
    """test_relocate_empty_clusters (:115-156): 2 empty clusters take the 2
    farthest points (10 and 9.5) in that order."""
    X = np.array([-10.0, -9.5, -9, -8.5, -8, -1, 1, 9, 9.5, 10], dtype=np.float32).reshape(-1, 1)
    C_old = np.array([[-10.0], [-10.0], [-10.0]], np.float32)
    q = R.fixed_q(X)
    lab = np.zeros(10, np.int32)
    xq = R.to_fixed(X, q)
    sums = np.zeros((3, 1), np.int64)
    sums[0] = xq.sum(0)
    cnt = np.array([10, 0, 0], np.int64)
    R.relocate(sums, cnt, R.far_candidates(X, C_old, lab, 0, 2), q)
    np.testing.assert_array_equal(cnt, [8, 1, 1])
    got = (sums.astype(np.float64) * 2.0 ** -q[0]).ravel()
    np.testing.assert_allclose(got, [-36.0, 10.0, 9.5])


def test_one_iteration_vs_python_reference():
    """test_k_means_1_iteration (:1000-1027): E, M, E against plain numpy."""
    X = np.random.RandomState(0).uniform(size=(100, 5)).astype(np.float32)
    init = X[:5].copy()
    d = ((X[:, None, :].astype(np.float64) - init[None].astype(np.float64)) ** 2).sum(-1)
    lab = d.argmin(1)
    newc = np.stack([X[lab == j].mean(0) for j in range(5)]).astype(np.float32)
    d2 = ((X[:, None, :].astype(np.float64) - newc[None].astype(np.float64)) ** 2).sum(-1)
    r = R.lloyd_fit(X, init, max_iter=1)
    np.testing.assert_array_equal(r["labels"], d2.argmin(1))
    np.testing.assert_allclose(r["centers"], newc, rtol=1e-6)


@pytest.mark.parametrize("d", [1, 2, 3, 4])
def test_numpy_and_c_restatements_agree(d):
    X = R.splitmix_uniform(30_000, d, 9) * np.float32(7) - np.float32(3)
    C = X[R.init_indices(30_000, 97)]
    q = R.fixed_q(X)
    old = np.random.default_rng(0).integers(-1, 97, 30_000).astype(np.int32)
    a = R.local_stats(X, C, old, q)
    b = cref.lloyd_stats(X, C, q, old, nthreads=4)
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[2], b[2])
    assert a[3] == b[3]


def test_sharded_fit_is_identical():
    X = R.splitmix_uniform(20_000, 3, 4)
    C0 = X[R.init_indices(20_000, 40)]
    a = R.lloyd_fit(X, C0, max_iter=12)
    b = R.lloyd_fit(X, C0, max_iter=12, shards=5)
    np.testing.assert_array_equal(a["labels"], b["labels"])
    np.testing.assert_array_equal(a["centers"], b["centers"])
    assert a["changed"] == b["changed"]


def test_fixed_point_bounds():
    X = np.array([[0.999999, -1500.0, 3e-9], [-0.5, 1499.9, 0.0]], np.float32)
    q = R.fixed_q(X)
    xq = R.to_fixed(X, q)
    assert np.all(np.abs(xq) < 2 ** R.QBITS)
    from pcm_amd.fixed import fixed_q as product_q
    np.testing.assert_array_equal(product_q(np.abs(X).max(0)), q)


def test_splitmix_deterministic_and_uniform():
    a = R.splitmix_uniform(1000, 3, 5)
    b = R.splitmix_uniform(10, 3, 5, start=500)
    np.testing.assert_array_equal(a[500:510], b)
    assert 0.0 <= a.min() and a.max() < 1.0
    assert abs(float(a.mean()) - 0.5) < 0.02


def test_relocation_donor_emptied_is_not_refilled():
    """The empty list is fixed before moves (_k_means_common.pyx:177-178): the
    donor of the farthest point (cluster 2, a singleton) becomes empty and must
    take the largest cluster's centre, not another point."""
    X = np.array([[0.0], [0.1], [0.2], [100.0]], np.float32)
    C0 = np.array([[1000.0], [0.0], [90.0]], np.float32)
    q = R.fixed_q(X)
    lab, sums, cnt, _ = R.local_stats(X, C0, np.full(4, -1, np.int32), q)
    np.testing.assert_array_equal(cnt, [0, 3, 1])
    R.relocate(sums, cnt, R.far_candidates(X, C0, lab, 0, 1), q)
    np.testing.assert_array_equal(cnt, [1, 3, 0])
    Cn = R.average(sums, cnt, q, C0)
    assert Cn[0, 0] == np.float32(100.0)
    assert Cn[2, 0] == Cn[1, 0]
