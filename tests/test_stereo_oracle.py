"""CPU: the stereo oracles are pinned to the reference's own code.

tests/golden/stereo/*.npz were produced by running the reference's functions
(members/rafael/disparity/processing.py:94-115 photoconsistency_map,
disparity.py:229-250 left_right_consistency, and the plugin.py:147-192 cloud
assembly block) on synthetic inputs -- see tests/golden/make_stereo_golden.py.
"""
import os

import numpy as np
import pytest

from oracle import cloud_ref, consistency_ref as CR

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "stereo")


@pytest.mark.parametrize("i", [0, 1, 2])
def test_consistency_oracle_equals_reference(i):
    g = np.load(os.path.join(GOLD, "consistency.npz"))
    left, right, ld, rd = g[f"left{i}"], g[f"right{i}"], g[f"ld{i}"], g[f"rd{i}"]
    np.testing.assert_array_equal(CR.photoconsistency_map(left, right, ld, -144), g[f"photo{i}"])
    np.testing.assert_array_equal(CR.left_right_consistency(ld, rd, -144), g[f"lr{i}"])


@pytest.mark.parametrize("i", [0, 1])
def test_cloud_oracle_equals_reference_block(i):
    g = np.load(os.path.join(GOLD, "cloud.npz"))
    pts, hn, nrm = cloud_ref.assemble(g[f"disp{i}"], g[f"valid{i}"])
    np.testing.assert_array_equal(pts, g[f"points{i}"])
    np.testing.assert_array_equal(hn, g[f"hnorm{i}"])
    np.testing.assert_array_equal(nrm, g[f"normal{i}"])


# ---------------------------------------------------------------- GPU (row f3)
@pytest.fixture(scope="module")
def gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pcm_amd
    return torch, pcm_amd


@pytest.mark.gpu
@pytest.mark.parametrize("i", [0, 1, 2])
def test_gpu_consistency_equals_reference(gpu, i):
    torch, pcm = gpu
    g = np.load(os.path.join(GOLD, "consistency.npz"))
    left, right, ld, rd = g[f"left{i}"], g[f"right{i}"], g[f"ld{i}"], g[f"rd{i}"]
    np.testing.assert_array_equal(pcm.photoconsistency_map(left, right, ld, -144), g[f"photo{i}"])
    np.testing.assert_array_equal(pcm.left_right_consistency(ld, rd, -144), g[f"lr{i}"])
    out, mask = pcm.left_right_consistency(ld, rd, -144, threshold=3)
    np.testing.assert_array_equal(mask, g[f"lr{i}"] < 3)
    # float64 images, device tensors in / out
    t = pcm.photoconsistency_map(torch.from_numpy(left.astype(np.float64)).cuda(),
                                 torch.from_numpy(right.astype(np.float64)).cuda(), torch.from_numpy(ld).cuda(), -144)
    np.testing.assert_array_equal(t.cpu().numpy(), g[f"photo{i}"])


@pytest.mark.gpu
def test_gpu_consistency_large_and_edges(gpu):
    """4k-wide rows, every undefined rule, min_disp boundary, integer rounding ties."""
    torch, pcm = gpu
    rng = np.random.default_rng(30)
    H, W = 300, 4100
    left = rng.uniform(0, 255, (H, W)).astype(np.float32)
    right = rng.uniform(0, 255, (H, W)).astype(np.float32)
    ld = np.round(rng.uniform(-160, 40, (H, W)) * 2) / 2          # many exact .5 values
    ld[rng.random((H, W)) < 0.03] = np.nan
    ld[:, 0] = -144.0                                               # == min_disp: defined
    ld[:, 1] = np.nextafter(-144.0, -np.inf)                        # just below: undefined
    ld[5, :] = np.inf
    ld[6, :] = -np.inf
    rd = -ld + rng.normal(0, 1.5, (H, W))
    np.testing.assert_array_equal(pcm.photoconsistency_map(left, right, ld, -144),
                                  CR.photoconsistency_map(left, right, ld, -144))
    np.testing.assert_array_equal(pcm.left_right_consistency(ld, rd, -144, 80),
                                  CR.left_right_consistency(ld, rd, -144, 80))
