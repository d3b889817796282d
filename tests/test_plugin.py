"""CPU plumbing of the drop-in plugin (SURVEY config 1: ~10k-point synthetic
cloud, K=8, no GPU).  The K-means backend is injected: the oracle here (the
product has no CPU fallback); the GPU path is tests/test_gpu_parity.py."""
import inspect

import numpy as np
import pytest

import pcm_amd
from fake_pipeline import SyntheticPairExtractor
from oracle import lloyd_ref as R


def oracle_fit(X, C0, max_iter, tol_abs):
    r = R.lloyd_fit(X, C0, max_iter=max_iter, tol=tol_abs)
    return r["labels"], r["centers"], r["inertia"], r["n_iter"]


def test_contract_matches_reference_component():
    p = pcm_amd.HeightMapExtractor()
    assert p.name == "Multi-day 3D Point Cloud" and "3D Point Cloud" in p.name   # viewer.py:475
    assert p.requires_image is False and p.requires_viewer is False
    sig = inspect.signature(p.run)
    assert list(sig.parameters) == ["kml_path", "is_debug_mode", "is_debug_pair", "is_one_random_pair", "n"]
    assert [sig.parameters[k].default for k in list(sig.parameters)[1:]] == [True, False, True, 10]


def test_config1_plumbing_cpu():
    base = SyntheticPairExtractor(n_pairs=1, shape=(100, 100))   # ~9k valid points
    plugin = pcm_amd.HeightMapExtractor(base=base, n_clusters=8, max_iter=300, tol=1e-4, fit=oracle_fit)
    layers = plugin.run("roi.kml", n=1)
    assert all(isinstance(l, tuple) and len(l) == 3 for l in layers)
    names = [l[1]["name"] for l in layers]
    assert names[-2:] == ["[Multi-day 3D Point Cloud] Fused K-means Centroids",
                          "[Multi-day 3D Point Cloud] Fused 3D Point Cloud"]
    cent, cloud = layers[-2], layers[-1]
    assert cent[2] == "points" and cent[0].shape == (8, 3)
    assert cloud[0].shape[0] == plugin.last_result["n_points"] > 8000
    lab = cloud[1]["properties"]["cluster"]
    assert lab.shape == (cloud[0].shape[0],) and lab.max() < 8
    # the result equals a direct oracle fit of the same fused cloud
    X = cloud[0].astype(np.float32)
    ref = R.lloyd_fit(X, X[R.init_indices(X.shape[0], 8)], max_iter=300,
                      tol=float(np.mean(np.var(X.astype(np.float64), axis=0)) * 1e-4))
    np.testing.assert_array_equal(lab, ref["labels"])
    np.testing.assert_array_equal(cent[0].astype(np.float32), ref["centers"])


def test_multi_pair_fusion_keeps_reference_layers():
    base = SyntheticPairExtractor(n_pairs=3, shape=(60, 80))
    plugin = pcm_amd.HeightMapExtractor(base=base, n_clusters=16, fit=oracle_fit)
    layers = plugin.run("roi.kml")
    ref_layers = base.run("roi.kml")
    assert len(layers) == len(ref_layers) + 2
    assert sum(l[0].shape[0] for l in ref_layers if l[2] == "points") == layers[-1][0].shape[0]


def test_errors_become_error_layer():
    def boom(*a, **k):
        raise RuntimeError("HIP extension missing")
    plugin = pcm_amd.HeightMapExtractor(base=SyntheticPairExtractor(), fit=boom)
    out = plugin.run("roi.kml")
    assert len(out) == 1 and out[0][2] == "image" and out[0][1]["name"].startswith("Error:")


def test_base_error_layer_passes_through():
    plugin = pcm_amd.HeightMapExtractor(base=SyntheticPairExtractor(fail=True), fit=oracle_fit)
    out = plugin.run("roi.kml")
    assert out[0][1]["name"] == "Error: synthetic failure"


def test_gpu_path_fails_loudly_without_device():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    plugin = pcm_amd.HeightMapExtractor(base=SyntheticPairExtractor(n_pairs=1, shape=(40, 40)), n_clusters=4)
    out = plugin.run("roi.kml")
    assert out[0][1]["name"].startswith("Error:")


# ---------------------------------------------------------------- GPU-stages path (rows a1-a4 / f2 / f4)
def oracle_assemble(disparity, validity):
    from oracle import cloud_ref
    pts, hn, _ = cloud_ref.assemble(disparity, validity)
    return pts, hn


def test_stages_path_layers_and_fusion_cpu(tmp_path):
    from fake_pipeline import SyntheticStages
    stages = SyntheticStages(n_pairs=2, shape=(70, 90))
    out = tmp_path / "fused.npz"
    plugin = pcm_amd.HeightMapExtractor(stages=stages, n_clusters=12, fit=oracle_fit, _assemble=oracle_assemble,
                                        export_path=str(out))
    layers = plugin.run("roi.kml")
    names = [l[1]["name"].replace("[Multi-day 3D Point Cloud] ", "") for l in layers]
    per_pair = ["Input Left", "Disparity", "Photoconsistency", "Invalid Mask", "3D Point Cloud"]   # plugin.py:119-233
    assert names == per_pair * 2 + ["Fused K-means Centroids", "Fused 3D Point Cloud"]
    clouds = [l[0] for l in layers if l[2] == "points" and l[1]["name"].endswith("] 3D Point Cloud")]
    X = np.concatenate(clouds).astype(np.float32)
    ref = R.lloyd_fit(X, X[R.init_indices(X.shape[0], 12)], max_iter=300,
                      tol=float(np.mean(np.var(X.astype(np.float64), axis=0)) * 1e-4))
    np.testing.assert_array_equal(layers[-1][1]["properties"]["cluster"], ref["labels"])
    # the Disparity image holds h_norm at the valid pixels (normalise_for_display of the relative heights)
    disp_img, pts, hn = layers[1][0], layers[4][0], layers[4][1]["properties"]["height"]
    np.testing.assert_array_equal(disp_img[pts[:, 1].astype(int), pts[:, 2].astype(int)], hn)
    assert np.isnan(disp_img).sum() == disp_img.size - pts.shape[0]
    # f4: the on-disk fused cloud
    f = pcm_amd.plugin.load_fused(str(out))
    np.testing.assert_array_equal(f["cluster"], ref["labels"])
    np.testing.assert_array_equal(f["points"], X.astype(np.float64))
    assert f["centers"].shape == (12, 3) and int(f["counts"].sum()) == X.shape[0]


def test_stages_error_becomes_error_layer():
    from fake_pipeline import SyntheticStages
    plugin = pcm_amd.HeightMapExtractor(stages=SyntheticStages(fail_at=1), fit=oracle_fit, _assemble=oracle_assemble)
    out = plugin.run("roi.kml")
    assert len(out) == 1 and out[0][1]["name"] == "Error: synthetic stereo failure"


def test_reference_error_layers():
    """plugin.py:77-79 / 89-91: a missing image and a failed crop return np.zeros((100, 100))
    named "error: image not found" / "error: <msg>"; other failures np.ones named "Error: <msg>"."""
    from fake_pipeline import SyntheticStages
    out = pcm_amd.HeightMapExtractor(stages=SyntheticStages(fail="image"), fit=oracle_fit).run("roi.kml")
    assert len(out) == 1 and out[0][1] == {"name": "error: image not found"} and out[0][2] == "image"
    assert out[0][0].shape == (100, 100) and not out[0][0].any()
    out = pcm_amd.HeightMapExtractor(stages=SyntheticStages(fail="crop"), fit=oracle_fit).run("roi.kml")
    assert out[0][1] == {"name": "error: KML region outside the image"} and not out[0][0].any()
    st = SyntheticStages(fail_at=0)
    out = pcm_amd.HeightMapExtractor(stages=st, fit=oracle_fit, _assemble=oracle_assemble).run("roi.kml")
    assert out[0][1] == {"name": "Error: synthetic stereo failure"} and out[0][0].shape == (100, 100)
    assert (out[0][0] == 1).all() and st.logged[-1].startswith("Error: synthetic stereo failure")


def test_stages_log_added_layers():
    from fake_pipeline import SyntheticStages
    st = SyntheticStages(n_pairs=1, shape=(40, 50))
    layers = pcm_amd.HeightMapExtractor(stages=st, n_clusters=4, fit=oracle_fit, _assemble=oracle_assemble).run("k")
    assert st.logged == [f"Added {len(layers)} layers to Napari"]    # plugin.py:234


@pytest.mark.gpu
def test_gpu_stages_path_device_fusion():
    """GPU cloud assembly on the plugin path (no host round trip into the K-means):
    the fused labels equal an oracle fit of the assembled clouds the layers show."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from fake_pipeline import SyntheticStages
    plugin = pcm_amd.HeightMapExtractor(stages=SyntheticStages(n_pairs=3, shape=(120, 150)), n_clusters=64,
                                        max_iter=40, tol=0.0)
    layers = plugin.run("roi.kml")
    assert layers[-1][1]["name"].endswith("Fused 3D Point Cloud"), layers[0][1]["name"]
    clouds = [l[0] for l in layers if l[2] == "points" and l[1]["name"].endswith("] 3D Point Cloud")]
    X = np.concatenate(clouds).astype(np.float32)
    ref = R.lloyd_fit(X, X[R.init_indices(X.shape[0], 64)], max_iter=40, fast=True)
    np.testing.assert_array_equal(layers[-1][1]["properties"]["cluster"], ref["labels"])
    np.testing.assert_array_equal(layers[-2][0].astype(np.float32), ref["centers"])
    # each pair's cloud is the GPU assembly of that pair (= the oracle to float64 rounding)
    from oracle import cloud_ref
    st = SyntheticStages(n_pairs=3, shape=(120, 150))
    for pp, cl in zip(st.pairs("roi.kml"), clouds):
        ref_pts, _, _ = cloud_ref.assemble(pp.disparity, pp.validity)
        np.testing.assert_array_equal(cl[:, 1:], ref_pts[:, 1:])
        np.testing.assert_allclose(cl[:, 0], ref_pts[:, 0], rtol=1e-9, atol=1e-9)


def _reference_message(fn):
    """The text of the exception the reference's own numpy expression raises."""
    try:
        fn()
    except IndexError as e:
        return str(e)
    raise AssertionError("expected IndexError")


@pytest.mark.parametrize("m", [0, 1, 2])
def test_too_few_valid_pixels_is_the_reference_error(m):
    """plugin.py:164-165: ``Vh[2]`` of the thin SVD of fewer than 3 valid pixels raises
    IndexError; plugin.py:236-241 turns the whole run into that one "Error: <msg>" layer."""
    from fake_pipeline import SyntheticStages
    msg = _reference_message(lambda: np.linalg.svd(np.zeros((m, 3)), full_matrices=False)[2][2])
    st = SyntheticStages(n_pairs=2, shape=(40, 50), n_valid=(1, m))
    out = pcm_amd.HeightMapExtractor(stages=st, n_clusters=4, fit=oracle_fit, _assemble=oracle_assemble).run("k")
    assert len(out) == 1 and out[0][1] == {"name": f"Error: {msg}"} and (out[0][0] == 1).all()
    assert st.logged[-1].startswith(f"Error: {msg}")


def test_three_valid_pixels_assemble():
    from fake_pipeline import SyntheticStages
    st = SyntheticStages(n_pairs=1, shape=(40, 50), n_valid=(0, 3))
    out = pcm_amd.HeightMapExtractor(stages=st, n_clusters=2, fit=oracle_fit, _assemble=oracle_assemble).run("k")
    assert out[-1][1]["name"].endswith("Fused 3D Point Cloud") and out[-1][0].shape == (3, 3)


def test_no_positive_photoconsistency_is_the_reference_error():
    """utils.py:12 via plugin.py:195-196: np.percentile of the empty positive-photoconsistency
    selection raises IndexError; the run becomes that "Error: <msg>" layer."""
    from fake_pipeline import SyntheticStages
    msg = _reference_message(lambda: np.percentile(np.zeros(0), [2, 98]))
    st = SyntheticStages(n_pairs=2, shape=(40, 50), dark_at=1)
    out = pcm_amd.HeightMapExtractor(stages=st, n_clusters=4, fit=oracle_fit, _assemble=oracle_assemble).run("k")
    assert len(out) == 1 and out[0][1] == {"name": f"Error: {msg}"} and (out[0][0] == 1).all()


@pytest.mark.gpu
@pytest.mark.parametrize("m", [0, 2])
def test_gpu_assembly_too_few_valid_pixels(m):
    """The product's GPU assembly raises the reference's IndexError (plugin.py:164-165)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from fake_pipeline import SyntheticStages
    msg = _reference_message(lambda: np.linalg.svd(np.zeros((m, 3)), full_matrices=False)[2][2])
    out = pcm_amd.HeightMapExtractor(stages=SyntheticStages(n_pairs=1, shape=(40, 50), n_valid=(0, m)),
                                     n_clusters=4).run("k")
    assert len(out) == 1 and out[0][1] == {"name": f"Error: {msg}"}
