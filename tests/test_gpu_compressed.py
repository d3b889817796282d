"""GPU: the compressed point stream of k_lloyd1 is lossless.

Tiles whose three axes are single-signed and whose delta widths sum to <= 64
bits are streamed as 8-byte records and decoded to the exact fp32 values.
Config-scale grids (32^3 cells) make most tiles compressible; here a dense
grid is forced on small clouds (PCM_CELL_TARGET, a tuning knob read at every
layout) so that every case has compressed tiles -- uniform, all-negative axes,
mixed-sign axes (raw tiles beside compressed ones), pixel-unit height-map
coordinates, exact duplicates -- and the fit must equal the oracle bit for
bit.  A run with compression disabled (PCM_XZ=0, read once per process: here
the number of compressed points) is not needed: the oracle is the reference.
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


def _clouds():
    rng = np.random.default_rng(11)
    n = 400_000
    u = R.splitmix_uniform(n, 3, 31)
    neg = u - np.float32(2.0)                                   # every axis negative
    mixed = u - np.float32(0.5)                                 # axes straddle 0: raw tiles near the planes
    yy = rng.integers(0, 1500, n).astype(np.float32)
    xx = rng.integers(0, 2200, n).astype(np.float32)
    zz = (8 * np.sin(xx / 230.0) + 5 * np.cos(yy / 170.0) + rng.normal(0, 0.3, n)).astype(np.float32)
    pix = np.stack([zz - zz.min(), yy, xx], 1).astype(np.float32)   # plugin.py:192 column order z, y, x
    dup = u.copy()
    dup[1000:3000] = dup[1000]
    return {"uniform": u, "negative": neg, "mixed": mixed, "pixel": pix, "dups": dup}


@pytest.mark.parametrize("name", ["uniform", "negative", "mixed", "pixel", "dups"])
def test_compressed_tiles_bitwise(pcm, name, monkeypatch):
    X = _clouds()[name]
    n = X.shape[0]
    C0 = X[R.init_indices(n, 96)]
    monkeypatch.setenv("PCM_CELL_TARGET", "20000")          # ~20 points per cell: narrow tiles
    from pcm_amd.engine import Engine
    from pcm_amd import lloyd
    eng = Engine(3, 96, torch.float32, max_iter=12)
    Xt = torch.from_numpy(X).cuda()
    lloyd.prepare(eng, Xt, lloyd.LOCAL)
    sb = eng.stream_bytes()
    assert 0 < sb["compressed_points"] <= n, sb
    if name == "mixed":
        assert sb["compressed_points"] < n                  # sign-straddling tiles stay raw
    assert sb["bytes"] == pytest.approx(8.0 * sb["compressed_points"] + 12.0 * (n - sb["compressed_points"]))
    res = pcm.lloyd_fit(Xt, torch.from_numpy(C0).cuda(), max_iter=12, tol=0.0, engine=eng)
    torch.cuda.synchronize()
    ref = R.lloyd_fit(X, C0, max_iter=12, tol=0.0, fast=True)
    np.testing.assert_array_equal(res.labels.cpu().numpy(), ref["labels"])
    np.testing.assert_array_equal(res.centers.cpu().numpy(), ref["centers"])
    assert res.n_iter == ref["n_iter"] and res.inertia == ref["inertia"]
