"""Per-pair cloud assembly.

CPU: the restatement oracle/cloud_ref.py equals the test pipeline's copy of
plugin.py:147-192 (tests/fake_pipeline.pair_cloud) exactly.  GPU:
``pcm_amd.assemble_cloud`` (HIP kernels through the C ABI) equals the oracle to
float64 rounding (the plane comes from a covariance eigen-solve instead of an
SVD, and sums run in another order): 1e-9 relative of the coordinate scale.
"""
import numpy as np
import pytest

from oracle import cloud_ref as CR


def synthetic_disparity(H, W, seed, invalid_frac=0.1):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W]
    disp = -16.0 * (8 * np.sin(xx / 23.0) + 5 * np.cos(yy / 17.0) + 0.02 * xx + rng.normal(0, 0.3, (H, W)))
    disp[rng.random((H, W)) < 0.02] = np.nan                    # WLS holes
    disp[rng.random((H, W)) < 0.01] = -16.0 * 1e4               # sentinel values beyond MAX_DISP/2
    validity = rng.random((H, W)) > invalid_frac
    return disp, validity


def test_oracle_matches_pipeline_copy():
    import fake_pipeline
    disp, validity = synthetic_disparity(90, 120, 1)
    pts, hn, _ = CR.assemble(disp, validity)
    h = -disp / 16.0
    valid = np.isfinite(h) & (np.abs(h) <= 144) & validity
    pts2, hn2 = fake_pipeline.pair_cloud(h, valid)
    np.testing.assert_array_equal(pts, pts2)
    np.testing.assert_array_equal(hn, hn2)


@pytest.fixture(scope="module")
def gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pcm_amd
    return pcm_amd


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,seed,frac", [(90, 120, 1, 0.1), (300, 257, 2, 0.3), (1000, 1000, 3, 0.05),
                                           (7, 5, 4, 0.0)])
def test_gpu_matches_oracle(gpu, H, W, seed, frac):
    disp, validity = synthetic_disparity(H, W, seed, frac)
    ref_pts, ref_hn, ref_n = CR.assemble(disp, validity)
    pts, hn, n = gpu.assemble_cloud(disp, validity)
    assert pts.shape == ref_pts.shape
    np.testing.assert_array_equal(pts[:, 1:], ref_pts[:, 1:])          # y, x: exact (np.where order)
    np.testing.assert_allclose(n, ref_n, rtol=0, atol=1e-9)
    scale = max(1.0, float(np.abs(ref_pts[:, 0]).max()))
    np.testing.assert_allclose(pts[:, 0], ref_pts[:, 0], rtol=0, atol=1e-9 * scale)
    np.testing.assert_allclose(hn, ref_hn, rtol=0, atol=1e-9)


@pytest.mark.gpu
def test_gpu_no_validity_and_empty(gpu):
    disp, _ = synthetic_disparity(64, 64, 5)
    ref_pts, _, _ = CR.assemble(disp, None)
    pts, _, _ = gpu.assemble_cloud(disp)
    np.testing.assert_array_equal(pts[:, 1:], ref_pts[:, 1:])
    # no valid pixel: the reference's plane fit raises this IndexError (plugin.py:164-165)
    with pytest.raises(IndexError, match="index 2 is out of bounds for axis 0 with size 0"):
        gpu.assemble_cloud(np.full((8, 8), np.nan))


@pytest.mark.gpu
@pytest.mark.parametrize("i", [0, 1])
def test_gpu_matches_reference_block(i):
    """GPU assembly vs the reference's own plugin.py:147-192 block (golden,
    tests/golden/make_stereo_golden.py): y, x exact; z, h_norm, normal to 1e-9."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import os
    import pcm_amd
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "stereo", "cloud.npz"))
    pts, hn, nrm = pcm_amd.assemble_cloud(g[f"disp{i}"], g[f"valid{i}"])
    ref = g[f"points{i}"]
    assert pts.shape == ref.shape
    np.testing.assert_array_equal(pts[:, 1:], ref[:, 1:])
    np.testing.assert_allclose(pts[:, 0], ref[:, 0], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(hn, g[f"hnorm{i}"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(nrm, g[f"normal{i}"], rtol=1e-9, atol=1e-12)
