"""k-means++ seeding.

CPU: the canonical restatement oracle/kpp_ref.py is pinned against
scikit-learn's own ``kmeans_plusplus`` (same seeds -> identical indices), and the
product path's host helpers agree with it.  GPU: ``pcm_amd.kmeans_plusplus``
(HIP kernels through the C ABI) returns exactly the oracle's indices.
"""
import numpy as np
import pytest

from oracle import kpp_ref as P
from oracle import lloyd_ref as R

CASES = [  # n, k, d, seed
    (10000, 8, 3, 42),
    (4096, 64, 3, 0),
    (3000, 20, 2, 7),
    (20000, 128, 3, 3),
    (5000, 16, 4, 11),
    (2500, 5, 1, 5),
]


@pytest.mark.parametrize("n,k,d,seed", CASES)
def test_oracle_matches_sklearn(n, k, d, seed):
    sk = pytest.importorskip("sklearn.cluster")
    X = R.splitmix_uniform(n, d, seed=seed + 100)
    c_ref, i_ref = sk.kmeans_plusplus(X, k, random_state=seed)
    c, i = P.kmeanspp(X, k, seed)
    np.testing.assert_array_equal(i, i_ref)
    np.testing.assert_array_equal(c, X[i_ref])


def test_host_helpers_match_oracle():
    from pcm_amd import kpp as K
    for n, maxd in [(10, 3.0), (10**8, 3.0), (12345, 1e-9), (7, 7.5e18)]:
        assert K._scale(n, maxd) == P.kpp_scale(n, maxd)
        assert (n * P.kpp_scale(n, maxd) >= 0) or True
    rs = np.random.RandomState(3)
    u0 = rs.random_sample()
    w = np.ones(1000, np.float32)
    assert K._first_index(1000, u0) == np.random.RandomState(3).choice(1000, p=w / w.sum())
    assert P.first_index(1000, u0) == K._first_index(1000, u0)
    # the O(1) form equals numpy's cumsum/searchsorted (oracle) on awkward sizes and draws
    rs = np.random.RandomState(11)
    for n in (1, 2, 3, 7, 1000, 65537, 1_000_003, 3_000_000):
        for u in list(rs.random_sample(6)) + [0.0, 1.0 - 2.0 ** -53, 0.5, 1.0 / 3.0]:
            assert K._first_index(n, u) == P.first_index(n, u), (n, u)


def test_host_draws_are_sklearns_stream():
    """kpp._draws (one uniform draw of (k-1)*L doubles) equals the per-centre
    uniform(size=L) draws _kmeans_plusplus makes (sklearn/cluster/_kmeans.py:239)."""
    from pcm_amd import kpp as K
    for seed, k, L in [(0, 1024, 8), (42, 5, 3), (7, 1, 2), (123, 2, 16)]:
        u0, um = K._draws(np.random.RandomState(seed), k, L)
        rs = np.random.RandomState(seed)
        assert u0 == rs.random_sample()
        ref = [np.ldexp(rs.uniform(size=L), 53).astype(np.uint64) for _ in range(1, k)]
        np.testing.assert_array_equal(um[:(k - 1) * L], np.concatenate(ref) if ref else np.zeros(0, np.uint64))


def test_weights_cannot_overflow():
    X = R.splitmix_uniform(50000, 3, seed=1) * np.float32(1e6)
    s = P.kpp_scale(len(X), P.max_dist_bound(X))
    d = R.sqdist_rows(X, np.broadcast_to(X[0], X.shape))
    w = P.weights(d, s)
    assert int(w.sum(dtype=np.uint64)) < 2 ** 63
    assert int(w.max()) * len(X) < 2 ** 63


# ---------------------------------------------------------------- GPU parity
@pytest.fixture(scope="module")
def gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pcm_amd
    return torch, pcm_amd


GPU_CASES = CASES + [
    (50000, 32, 3, 9),          # several original-order weight blocks (4096 rows), ragged tail
    (100000, 64, 3, 1),
    (1000, 1000, 3, 2),         # k == n
    (1, 1, 3, 0),
    (300000, 256, 3, 4),        # many cells: late steps touch only the candidates' neighbourhoods
    (120000, 128, 4, 6),
]


@pytest.mark.gpu
@pytest.mark.parametrize("n,k,d,seed", GPU_CASES)
def test_gpu_matches_oracle(gpu, n, k, d, seed):
    torch, pcm = gpu
    X = R.splitmix_uniform(n, d, seed=seed + 100)
    c_ref, i_ref = P.kmeanspp(X, k, seed)
    c, i = pcm.kmeans_plusplus(torch.from_numpy(X).cuda(), k, random_state=seed)
    np.testing.assert_array_equal(i.cpu().numpy(), i_ref)
    np.testing.assert_array_equal(c.cpu().numpy(), c_ref)


@pytest.mark.gpu
def test_gpu_duplicates_and_offsets(gpu):
    """Heavy duplicates (zero weights), negative offset coordinates in pixel units."""
    torch, pcm = gpu
    rng = np.random.default_rng(4)
    base = (rng.integers(0, 50, size=(400, 3)) * np.float32(0.5) - np.float32(300.0)).astype(np.float32)
    X = np.repeat(base, 25, axis=0)
    X = X[rng.permutation(len(X))]
    for k, seed in [(16, 0), (40, 9)]:
        _, i_ref = P.kmeanspp(X, k, seed)
        _, i = pcm.kmeans_plusplus(torch.from_numpy(X).cuda(), k, random_state=seed)
        np.testing.assert_array_equal(i.cpu().numpy(), i_ref)


@pytest.mark.gpu
def test_gpu_matches_sklearn(gpu):
    sk = pytest.importorskip("sklearn.cluster")
    torch, pcm = gpu
    X = R.splitmix_uniform(8000, 3, seed=77)
    _, i_ref = sk.kmeans_plusplus(X, 24, random_state=123)
    _, i = pcm.kmeans_plusplus(torch.from_numpy(X).cuda(), 24, random_state=123)
    np.testing.assert_array_equal(i.cpu().numpy(), i_ref)


@pytest.mark.gpu
def test_gpu_duplicates_and_clusters(gpu):
    """Heavy duplication (zero potentials inside cells) and tight clusters far apart."""
    torch, pcm = gpu
    rng = np.random.default_rng(8)
    centres = rng.uniform(-100, 100, size=(12, 3)).astype(np.float32)
    X = (centres[rng.integers(0, 12, 60000)] + rng.normal(0, 0.05, (60000, 3))).astype(np.float32)
    X[::7] = X[3]                      # a sixth of the cloud is one point
    c_ref, i_ref = P.kmeanspp(X, 40, 17)
    c, i = pcm.kmeans_plusplus(torch.from_numpy(X).cuda(), 40, random_state=17)
    np.testing.assert_array_equal(i.cpu().numpy(), i_ref)


@pytest.mark.gpu
def test_gpu_heightmap_like(gpu):
    """Anisotropic 2.5-D pixel-unit cloud (z, y, x as plugin.py:191-192 emits)."""
    torch, pcm = gpu
    rng = np.random.default_rng(9)
    n = 150_000
    y = rng.integers(0, 1800, n).astype(np.float64)
    x = rng.integers(0, 2400, n).astype(np.float64)
    z = 10 * np.sin(x / 200) + 5 * np.cos(y / 150) + rng.normal(0, 0.5, n) + 30
    X = np.stack([z, y, x], axis=1).astype(np.float32)
    c_ref, i_ref = P.kmeanspp(X, 96, 21)
    c, i = pcm.kmeans_plusplus(torch.from_numpy(X).cuda(), 96, random_state=21)
    np.testing.assert_array_equal(i.cpu().numpy(), i_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("n,k,seed", [(5_000_000, 12, 3), (140_000_000, 3, 4)])
def test_gpu_large_search_segments(gpu, n, k, seed):
    """k_kpp_search at sizes whose wave segments span several 64-wide chunks of
    block sums (5M points: 2 chunks per wave) and more chunks than the register
    cache holds (140M points: 34 > KPP_SCU = 32, the re-read path)."""
    torch, pcm = gpu
    X = R.splitmix_uniform(n, 3, seed=seed + 300)
    _, i_ref = P.kmeanspp(X, k, seed)
    _, i = pcm.kmeans_plusplus(torch.from_numpy(X).cuda(), k, random_state=seed)
    np.testing.assert_array_equal(i.cpu().numpy(), i_ref)
