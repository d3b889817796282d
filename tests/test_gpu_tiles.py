"""GPU: tiles longer than TILE = 4096 points (round 5, DESIGN.md §4 "Big tiles").

Cells that are single-signed on every axis may hold tiles of up to TILE_BIG =
8192 points; the k_lloyd1 fold then reads each shared LDS word (<= 128 values of
one sign, |sum| < 2^32) as unsigned, or as a non-positive sum, instead of as
int32.  Cells that straddle 0 on some axis keep 4096-point tiles.  These clouds
put ~6k points in every cell (small K: few cells) with coordinates near the top
of the fixed-point range (|x| in [0.5, 1): trunc(x * 2^25) >= 2^24), so a word
holds sums close to 2^32: labels, centres, n_iter and inertia must equal the
oracle bit for bit.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import lloyd_ref as R  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pcm():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pcm_amd
    return pcm_amd


def _cloud(kind, n, d, seed=3):
    u = R.splitmix_uniform(n, d, seed)
    if kind == "pos":
        return np.ascontiguousarray(0.5 + 0.5 * u, dtype=np.float32)          # [0.5, 1)
    if kind == "neg":
        return np.ascontiguousarray(-(0.5 + 0.5 * u), dtype=np.float32)       # (-1, -0.5]
    if kind == "mixed":   # x >= 0, y <= 0, z straddles 0 (its middle cells keep 4096-point tiles)
        X = np.empty((n, d), np.float32)
        X[:, 0] = 0.5 + 0.5 * u[:, 0]
        X[:, 1] = -(0.5 + 0.5 * u[:, 1])
        X[:, 2:] = 2.0 * u[:, 2:] - 1.0
        return np.ascontiguousarray(X)
    raise ValueError(kind)


@pytest.mark.parametrize("kind,d,dt", [("pos", 3, torch.float32), ("neg", 3, torch.float32),
                                       ("mixed", 3, torch.float32), ("pos", 2, torch.float32),
                                       ("neg", 4, torch.float16), ("mixed", 4, torch.float16)])
def test_big_tiles_bitwise(pcm, kind, d, dt):
    n, k, iters = 1_500_000, 8, 12
    X = _cloud(kind, n, d)
    if dt == torch.float16:
        X = X.astype(np.float16).astype(np.float32)    # the values the fp16 engine sees
    C0 = X[R.init_indices(n, k)].copy()
    res = pcm.lloyd_fit(torch.from_numpy(X).cuda().to(dt), torch.from_numpy(C0).cuda(), max_iter=iters, tol=0.0)
    torch.cuda.synchronize()
    lay = res.layout
    per_cell = n / lay["ncells"]
    assert per_cell > 4096, lay                        # cells past the 4096-point cap
    if kind == "mixed":
        assert lay["ntiles"] > lay["ncells"], lay      # straddling cells were split
    else:
        assert lay["ntiles"] == lay["ncells"], lay     # one (big) tile per cell
    ref = R.lloyd_fit(X, C0, max_iter=iters, tol=0.0, fast=True)
    np.testing.assert_array_equal(res.labels.cpu().numpy(), ref["labels"])
    np.testing.assert_array_equal(res.centers.cpu().numpy(), ref["centers"])
    assert res.n_iter == ref["n_iter"] and float(res.inertia) == ref["inertia"]
