"""CPU: ``pcm_amd.pipeline.ReferenceStereoStages`` against a stand-in of the
reference package (TEST ONLY -- the real ``members.rafael.disparity`` needs
GDAL/OpenCV/rasterio/ASP and must not be imported).

The stand-in modules have the reference's module layout and names
(constants, disparity, pair_selector, preprocessing, processing, utils); their
``disparity_map`` resolves ``left_right_consistency`` / ``photoconsistency_map``
from its module globals, as ``disparity.py:157-161`` does.  Checked: the
gathers are the HIP drop-ins while ``disparity_map`` runs and the reference's
afterwards (also after an error), the run log ``TEMP/log.txt`` is written,
and missing images / failed crops map to the reference's error layers.
"""
import os
import sys
import types

import numpy as np
import pytest

import pcm_amd
from pcm_amd import pipeline


def _ref_lrc(left_disp, right_disp, min_disp, max_disp=80):
    return np.zeros(left_disp.shape)


def _ref_photo(left, right, left_disp, min_disp):
    return np.zeros(left_disp.shape)


@pytest.fixture
def fake_reference(tmp_path, monkeypatch):
    temp = str(tmp_path / "TEMP")
    wv3 = tmp_path / "WV3"
    wv3.mkdir()
    seen = {"gathers": [], "crop": 0, "fail_disparity": False, "fail_crop": False}

    pkg = {name: types.ModuleType(name) for name in
           ["members", "members.rafael", "members.rafael.disparity", "members.rafael.disparity.constants",
            "members.rafael.disparity.disparity", "members.rafael.disparity.pair_selector",
            "members.rafael.disparity.preprocessing", "members.rafael.disparity.processing",
            "members.rafael.disparity.utils"]}
    C = pkg["members.rafael.disparity.constants"]
    C.TEMP_PATH = temp
    C.WV3_PATH = str(wv3)
    C.TMP_STEREO_OUTPUT_PATH = temp + "/stereo_output"
    C.TMP_CROPPED_IMAGES_PATH = temp + "/cropped_images"
    C.TMP_DISPARITY_DEBUG_PATH = temp + "/disp_debug"
    C.PAIR_DECENT_RESULTS = [("a", "b")]

    class Img:
        def __init__(self, name, exists=True):
            self.filename, self.cropped_name = name, name + ".tif"
            self.path = str(wv3 / (name + ".NTF"))
            if exists:
                open(self.path, "w").close()

    class Pair:
        def __init__(self, a, b):
            self.img1, self.img2 = a, b

    state = {"pairs": [Pair(Img("a"), Img("b"))]}

    class PairSelector:
        def __init__(self, path):
            pass

        def discover_images(self):
            pass

        def select_pairs(self):
            return state["pairs"]

    pkg["members.rafael.disparity.pair_selector"].PairSelector = PairSelector

    def get_crop_area_from_kml(img, kml):
        if seen["fail_crop"]:
            raise ValueError("ROI outside the image")
        return (0, 0, 10, 10)

    def generate_cropped(img, out, name, area):
        seen["crop"] += 1

    pkg["members.rafael.disparity.preprocessing"].get_crop_area_from_kml = get_crop_area_from_kml
    pkg["members.rafael.disparity.preprocessing"].generate_cropped = generate_cropped
    pkg["members.rafael.disparity.processing"].generate_rectified = lambda pair, pid, out: out
    def open_tiff_file(path):
        if seen.get("missing_crop") and os.path.basename(path) == seen["missing_crop"]:
            raise FileNotFoundError(f"No such file: {path}")
        return np.ones((4, 4))

    pkg["members.rafael.disparity.utils"].open_tiff_file = open_tiff_file

    D = pkg["members.rafael.disparity.disparity"]
    D.left_right_consistency = _ref_lrc
    D.photoconsistency_map = _ref_photo

    def disparity_map(pair, pair_id, out, crop, dbg):
        g = D.__dict__     # what the reference body resolves at disparity.py:157-161
        seen["gathers"].append((g["left_right_consistency"], g["photoconsistency_map"]))
        if seen["fail_disparity"]:
            raise RuntimeError("SGBM failed")
        H, W = 30, 40
        yy, xx = np.mgrid[0:H, 0:W]
        disp = -16.0 * (3 * np.sin(xx / 7.0) + 2 * np.cos(yy / 5.0))
        return disp, np.ones((H, W), bool), np.full((H, W), 0.1)

    D.disparity_map = disparity_map
    for name, mod in pkg.items():
        monkeypatch.setitem(sys.modules, name, mod)
    return dict(seen=seen, state=state, temp=temp, Img=Img, Pair=Pair)


def _oracle_fit(X, C0, max_iter, tol_abs):
    from oracle import lloyd_ref as R
    r = R.lloyd_fit(X, C0, max_iter=max_iter, tol=tol_abs)
    return r["labels"], r["centers"], r["inertia"], r["n_iter"]


def _oracle_assemble(disparity, validity):
    from oracle import cloud_ref
    pts, hn, _ = cloud_ref.assemble(disparity, validity)
    return pts, hn


def _plugin(**kw):
    return pcm_amd.HeightMapExtractor(n_clusters=6, fit=_oracle_fit, _assemble=_oracle_assemble, **kw)


def test_gathers_rebound_during_disparity_map_and_restored(fake_reference):
    from pcm_amd import stereo
    D = sys.modules["members.rafael.disparity.disparity"]
    layers = _plugin().run("roi.kml", is_debug_mode=False)
    assert layers[-1][1]["name"].endswith("Fused 3D Point Cloud")
    (lrc, photo), = fake_reference["seen"]["gathers"]
    assert lrc is stereo.left_right_consistency and photo is stereo.photoconsistency_map
    assert D.left_right_consistency is _ref_lrc and D.photoconsistency_map is _ref_photo
    log = open(os.path.join(fake_reference["temp"], "log.txt")).read()
    assert log.startswith("3D Point Cloud started") and "Disparity map generated successfully" in log
    assert log.endswith(f"Added {len(layers)} layers to Napari")


def test_gathers_restored_after_error(fake_reference):
    fake_reference["seen"]["fail_disparity"] = True
    D = sys.modules["members.rafael.disparity.disparity"]
    out = _plugin().run("roi.kml")
    assert out[0][1] == {"name": "Error: SGBM failed"} and (out[0][0] == 1).all()
    assert D.left_right_consistency is _ref_lrc and D.photoconsistency_map is _ref_photo
    assert "Error: SGBM failed" in open(os.path.join(fake_reference["temp"], "log.txt")).read()


def test_numpy_gathers_kept_when_disabled(fake_reference):
    out = _plugin(stages=pipeline.ReferenceStereoStages(gpu_gathers=False)).run("roi.kml")
    assert out[-1][1]["name"].endswith("Fused 3D Point Cloud")
    assert fake_reference["seen"]["gathers"] == [(_ref_lrc, _ref_photo)]


def test_missing_image_and_failed_crop(fake_reference):
    fr = fake_reference
    fr["state"]["pairs"] = [fr["Pair"](fr["Img"]("a"), fr["Img"]("gone", exists=False))]
    out = _plugin().run("roi.kml")
    assert out == [] or (out[0][1] == {"name": "error: image not found"} and not out[0][0].any())
    assert len(out) == 1
    fr["state"]["pairs"] = [fr["Pair"](fr["Img"]("a"), fr["Img"]("b"))]
    fr["seen"]["fail_crop"] = True
    out = _plugin().run("roi.kml")
    assert len(out) == 1 and out[0][1] == {"name": "error: ROI outside the image"}
    assert out[0][0].shape == (100, 100) and not out[0][0].any()


def test_use_gpu_gathers_refcount():
    from pcm_amd import stereo
    m = types.ModuleType("fake_disparity")
    m.left_right_consistency, m.photoconsistency_map = _ref_lrc, _ref_photo
    with pipeline.use_gpu_gathers(m):
        with pipeline.use_gpu_gathers(m):
            assert m.left_right_consistency is stereo.left_right_consistency
        assert m.photoconsistency_map is stereo.photoconsistency_map     # still held by the outer user
    assert m.left_right_consistency is _ref_lrc and m.photoconsistency_map is _ref_photo


def test_debug_images_logged_and_missing_crop_is_an_error_layer(fake_reference):
    """plugin.py:120-131: the debug branch logs "Loading  basic cropped image for
    display..." and opens the cropped Input Left/Right unconditionally, so a
    missing crop raises and becomes the reference's "Error: ..." layer."""
    out = _plugin().run("roi.kml", is_debug_mode=True)
    names = [l[1]["name"] for l in out]
    assert any(n.endswith("Input Left") for n in names) and any(n.endswith("Input Right") for n in names)
    log = open(os.path.join(fake_reference["temp"], "log.txt")).read()
    assert "Loading  basic cropped image for display..." in log
    fake_reference["seen"]["missing_crop"] = "b.tif"
    out = _plugin().run("roi.kml", is_debug_mode=True)
    assert len(out) == 1 and out[0][1]["name"].startswith("Error: No such file") and (out[0][0] == 1).all()


def test_use_gpu_gathers_refcount_per_module():
    """Two modules rebound in interleaved blocks: each gets back its own originals
    (one shared count restored the wrong module)."""
    from pcm_amd import stereo
    a, b = types.ModuleType("fake_a"), types.ModuleType("fake_b")
    a.left_right_consistency, a.photoconsistency_map = _ref_lrc, _ref_photo
    b.photoconsistency_map = _ref_photo          # b lacks left_right_consistency
    ca, cb = pipeline.use_gpu_gathers(a), pipeline.use_gpu_gathers(b)
    ca.__enter__()
    cb.__enter__()
    assert b.left_right_consistency is stereo.left_right_consistency
    ca.__exit__(None, None, None)                # a restored while b is still rebound
    assert a.left_right_consistency is _ref_lrc and a.photoconsistency_map is _ref_photo
    assert b.photoconsistency_map is stereo.photoconsistency_map
    cb.__exit__(None, None, None)
    assert b.photoconsistency_map is _ref_photo and not hasattr(b, "left_right_consistency")
