"""GPU: crowded layouts (tile lists: csrc/pcm_kernels.hpp "crowded cells: tile lists", k_tile_cand) are exact.

Tight clusters put a whole cluster and its hundreds of centres into one grid
cell: the cell's list overflows CAPF (FULL) and, without tile lists, every
point of it scans all K centres.  A crowded layout orders each cell's points by
a Morton code of zlev bisections (compact tiles) and k_tile_cand builds a list
per tile of a FULL cell over the tile's exact point box.  Whatever the level
count -- detected from the occupancy sample, or forced with PCM_ZLEV (read at
every layout) -- the fit must equal the oracle bit for bit, and on these clouds
the tile lists must actually be used.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import lloyd_ref as R  # noqa: E402

pytestmark = pytest.mark.gpu

K = 256


@pytest.fixture(scope="module")
def pcm():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pcm_amd
    return pcm_amd


def _cloud(name, d=3):
    rng = np.random.default_rng(5)
    n = 240_000
    u = R.splitmix_uniform(n, d, 17)
    nc = 2 if name != "many" else 12
    cen = rng.random((nc, d)).astype(np.float32)
    cid = rng.integers(0, nc, n)
    X = (cen[cid] + rng.normal(0, 0.004, (n, d))).astype(np.float32)
    keep = u[:, 0] < 0.01                        # 1 % uniform background
    X[keep] = u[keep]
    if name == "negative":
        X = X - np.float32(3.0)
    if name == "dups":
        X[5000:9000] = X[5000]
    return np.ascontiguousarray(X)


@pytest.mark.parametrize("zlev", ["auto", "0", "2", "5"])
@pytest.mark.parametrize("name", ["clusters", "negative", "many", "dups"])
def test_crowded_bitwise(pcm, name, zlev, monkeypatch):
    X = _cloud(name)
    n = X.shape[0]
    C0 = X[R.init_indices(n, K)]
    if zlev == "auto":
        monkeypatch.delenv("PCM_ZLEV", raising=False)
    else:
        monkeypatch.setenv("PCM_ZLEV", zlev)
    from pcm_amd.engine import Engine
    from pcm_amd import lloyd
    eng = Engine(3, K, torch.float32, max_iter=12)
    Xt = torch.from_numpy(X).cuda()
    lloyd.prepare(eng, Xt, lloyd.LOCAL)
    res = pcm.lloyd_fit(Xt, torch.from_numpy(C0).cuda(), max_iter=12, tol=0.0, engine=eng)
    torch.cuda.synchronize()
    st = eng.candidate_stats()
    if zlev != "0":
        assert st.get("zlev", 0) > 0, st                 # detected (auto) or forced
        assert st["crowded_tiles"] > 0 and st["listed_tiles"] > 0, st   # long-list cells' tiles got their own lists
    else:
        assert "zlev" not in st
    ref = R.lloyd_fit(X, C0, max_iter=12, tol=0.0, fast=True)
    np.testing.assert_array_equal(res.labels.cpu().numpy(), ref["labels"])
    np.testing.assert_array_equal(res.centers.cpu().numpy(), ref["centers"])
    assert res.n_iter == ref["n_iter"] and res.inertia == ref["inertia"]


def test_crowded_2d_and_f16(pcm, monkeypatch):
    """D = 2 (two Morton bits per level) and fp16 points at D = 4 (four)."""
    monkeypatch.setenv("PCM_ZLEV", "3")
    from pcm_amd.engine import Engine
    from pcm_amd import lloyd
    for d, dt in ((2, torch.float32), (4, torch.float16)):
        X = _cloud("clusters", d)
        if dt == torch.float16:
            X = X.astype(np.float16).astype(np.float32)   # the values the fp16 engine sees
        n = X.shape[0]
        C0 = X[R.init_indices(n, K)]
        eng = Engine(d, K, dt, max_iter=10)
        Xt = torch.from_numpy(X).cuda().to(dt)
        lloyd.prepare(eng, Xt, lloyd.LOCAL)
        res = pcm.lloyd_fit(Xt, torch.from_numpy(C0).cuda(), max_iter=10, tol=0.0, engine=eng)
        torch.cuda.synchronize()
        assert eng.candidate_stats().get("zlev") == 3
        ref = R.lloyd_fit(X, C0, max_iter=10, tol=0.0, fast=True)
        np.testing.assert_array_equal(res.labels.cpu().numpy(), ref["labels"])
        np.testing.assert_array_equal(res.centers.cpu().numpy(), ref["centers"])


@pytest.mark.parametrize("name,zlev,k,expect", [
    ("many", "auto", 4096, "long"),       # tile lists of 257..1024 entries: LDS chunks, carried bd/bj
    ("clusters", "1", 4096, "allk"),      # one Morton level: a tile spans its whole cluster -> past 1024 -> all K
    ("clusters", "1", 1024, "any"),       # ~512 centres per cluster: lists past 256
])
def test_crowded_long_lists_and_allk_tiles(pcm, name, zlev, k, expect, monkeypatch):
    """the chunked crowded path of k_lloyd1 (tile lists longer than TLCAP = 256,
    all-K tiles staged through LDS in 256-centre chunks with the best distance carried
    across chunks, the direct-mapped LDS table whose j mod 256 collisions spill to global
    atomics) at K = 1024 and 4096, bitwise against the oracle; candidate_stats must show
    that the path ran."""
    X = _cloud(name)
    n = X.shape[0]
    C0 = X[R.init_indices(n, k)]
    if zlev == "auto":
        monkeypatch.delenv("PCM_ZLEV", raising=False)
    else:
        monkeypatch.setenv("PCM_ZLEV", zlev)
    from pcm_amd.engine import Engine
    from pcm_amd import lloyd
    eng = Engine(3, k, torch.float32, max_iter=8)
    Xt = torch.from_numpy(X).cuda()
    lloyd.prepare(eng, Xt, lloyd.LOCAL)
    res = pcm.lloyd_fit(Xt, torch.from_numpy(C0).cuda(), max_iter=8, tol=0.0, engine=eng)
    torch.cuda.synchronize()
    st = eng.candidate_stats()
    print(name, zlev, k, st)
    if expect == "long":
        assert st["long_tile_lists"] > 0 and st["tile_list_max"] > 256, st
    elif expect == "allk":
        assert st["allk_tiles"] > 0, st
    else:
        assert st["long_tile_lists"] + st["allk_tiles"] > 0, st
    ref = R.lloyd_fit(X, C0, max_iter=8, tol=0.0, fast=True)
    np.testing.assert_array_equal(res.labels.cpu().numpy(), ref["labels"])
    np.testing.assert_array_equal(res.centers.cpu().numpy(), ref["centers"])
    assert res.n_iter == ref["n_iter"] and res.inertia == ref["inertia"]
