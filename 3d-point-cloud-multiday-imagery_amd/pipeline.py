"""Per-pair stages of the reference plugin, with the cloud assembly on the GPU
(SURVEY.md §8 rows a1-a4 / f2).

The reference ``HeightMapExtractor.run`` (``members/rafael/disparity/plugin.py:36-243``)
does, per stereo pair: ASP rectification, SGBM/WLS disparity (OpenCV), then the
float64 NumPy cloud assembly of ``plugin.py:147-192`` and the per-pair layers of
``plugin.py:176-233``.  This module splits that loop at the assembly:

* ``ReferenceStereoStages.pairs(...)`` replays ``plugin.py:45-145`` with the
  reference's own functions (pair selection, KML crop, ASP rectification,
  ``disparity_map``; imported lazily, only inside the reference tree) and yields
  one ``PairProducts`` per pair -- the debug image layers it emits before the
  assembly, the disparity, its validity mask and the photoconsistency map;
* while ``disparity_map`` runs, its L/R-consistency and photoconsistency
  gathers (``disparity.py:157-161``, the names bound at ``disparity.py:7-9`` and
  defined at ``disparity.py:229-250`` / ``processing.py:94-115``) resolve to the
  HIP drop-ins of ``stereo.py`` (``use_gpu_gathers``, row f3);
* failures keep the reference's error layers: a missing image and a failed crop
  raise ``ImageNotFound`` / ``CropFailed``, which the plugin turns into
  ``(np.zeros((100, 100)), {"name": "error: ..."}, "image")``
  (``plugin.py:77-79, 89-91``); the run log goes to ``TEMP/log.txt``
  (``plugin.py:49-50, 234, 240``);
* ``pair_layers(...)`` rebuilds the per-pair layers of ``plugin.py:176-233``
  from the GPU assembly (``cloud.assemble_cloud_device``) -- the height-map
  image (``normalise_for_display`` of the relative heights equals the
  assembly's ``h_norm`` at valid pixels), photoconsistency, invalid mask and
  the 3D point cloud layer -- while the device copy of each cloud feeds the
  fused K-means without a host round trip.
"""
from __future__ import annotations

import contextlib
import os
import threading
from dataclasses import dataclass, field
from typing import Iterator, List

import numpy as np

PREFIX = "[Multi-day 3D Point Cloud]"
MASK_COLORMAP = {"colors": [[0.0, 0.0, 0.0, 0.0], [0.0, 0.0, 0.0, 1.0]], "name": "mask_blackout",
                 "interpolation": "linear"}


class ImageNotFound(FileNotFoundError):
    """A stereo image of a selected pair is missing (plugin.py:77-79)."""


class CropFailed(RuntimeError):
    """Cropping an image to the KML region failed (plugin.py:83-91); str() is the cause's message."""


GATHER_NAMES = ("left_right_consistency", "photoconsistency_map")
_gather_lock = threading.Lock()
_gather_users: dict = {}     # id(module) -> active use_gpu_gathers blocks on that module
_gather_saved: dict = {}     # id(module) -> {name: original binding} (names the module had)


@contextlib.contextmanager
def use_gpu_gathers(module):
    """Rebind ``module.left_right_consistency`` / ``module.photoconsistency_map``
    (the globals ``disparity_map`` resolves at ``disparity.py:157-161``) to the HIP
    drop-ins for the duration of the block; restored on exit (also on error).
    Reference-counted per module, so concurrent plugin runs share one binding and
    each module gets back exactly its own originals."""
    from . import stereo
    key = id(module)
    with _gather_lock:
        if _gather_users.get(key, 0) == 0:
            _gather_saved[key] = {name: getattr(module, name) for name in GATHER_NAMES if hasattr(module, name)}
            for name in GATHER_NAMES:
                setattr(module, name, getattr(stereo, name))
        _gather_users[key] = _gather_users.get(key, 0) + 1
    try:
        yield module
    finally:
        with _gather_lock:
            _gather_users[key] -= 1
            if _gather_users[key] == 0:
                del _gather_users[key]
                saved = _gather_saved.pop(key, {})
                for name in GATHER_NAMES:
                    if name in saved:
                        setattr(module, name, saved[name])
                    else:
                        delattr(module, name)


@dataclass
class PairProducts:
    disparity: np.ndarray                 # (H, W) SGBM/WLS disparity (x16 fixed point)
    validity: np.ndarray                  # (H, W) bool (disparity_map's final_defined)
    photoconsistency: np.ndarray          # (H, W) float64
    image_layers: List = field(default_factory=list)   # debug layers emitted before the assembly


def normalise_for_display(image: np.ndarray, mask: np.ndarray) -> np.ndarray:
    """``members/rafael/disparity/utils.py:9-14``: 2/98 percentiles of the masked
    values -> [0, 1] (host: a display helper, not on the K-means path)."""
    image = image.astype(float)
    p2, p98 = np.percentile(image[mask], [2, 98])
    return np.clip((image - p2) / (p98 - p2 + 1e-6), 0, 1)


def pair_layers(pp: PairProducts, points: np.ndarray, h_norm: np.ndarray) -> list:
    """Layers of plugin.py:176-233 for one pair from the assembled cloud (host copies)."""
    H, W = pp.disparity.shape
    y = points[:, 1].astype(np.int64)
    x = points[:, 2].astype(np.int64)
    height = np.full((H, W), np.nan)
    height[y, x] = h_norm                      # normalise_for_display(height_map, valid) at valid pixels
    layers = [(height, {"name": f"{PREFIX} Disparity", "colormap": "turbo", "scale": (1, 1)}, "image")]
    valid = pp.photoconsistency > 0            # plugin.py:195
    # no positive photoconsistency: np.percentile of an empty selection raises
    # IndexError inside normalise_for_display (utils.py:12 via plugin.py:196), as
    # in the reference, and the run becomes its "Error: <msg>" layer
    layers.append((normalise_for_display(pp.photoconsistency, valid),
                   {"name": f"{PREFIX} Photoconsistency", "colormap": "turbo", "scale": (1, 1)}, "image"))
    layers.append(((~valid).astype(np.float32), {"name": f"{PREFIX} Invalid Mask", "colormap": MASK_COLORMAP,
                                                   "scale": (1, 1), "contrast_limits": [0, 1]}, "image"))
    layers.append((points, {"name": f"{PREFIX} 3D Point Cloud", "size": 2, "properties": {"height": h_norm},
                            "scale": (1, 1, 1), "opacity": 0.8, "face_colormap": "turbo", "face_color": "height"},
                   "points"))
    return layers


class ReferenceStereoStages:
    """plugin.py:45-145 with the reference's functions (runs inside the reference tree).

    ``gpu_gathers``: run ``disparity_map``'s consistency gathers on the GPU
    (``use_gpu_gathers``); False keeps the reference's NumPy ones."""

    def __init__(self, gpu_gathers: bool = True):
        self.gpu_gathers = gpu_gathers
        self._log = None

    # plugin.py:49-50: the run log, TEMP/log.txt, opened once TEMP exists
    def log(self, msg: str):
        if self._log is not None:
            self._log.write(msg)

    def close_log(self):
        if self._log is not None:
            self._log.close()
            self._log = None

    def pairs(self, kml_path, is_debug_mode: bool = True, is_debug_pair: bool = False,
              is_one_random_pair: bool = True, n: int = 10) -> Iterator[PairProducts]:
        import shutil

        from members.rafael.disparity import constants as C  # type: ignore
        from members.rafael.disparity import disparity as dmod  # type: ignore
        from members.rafael.disparity.pair_selector import PairSelector  # type: ignore
        from members.rafael.disparity.preprocessing import generate_cropped, get_crop_area_from_kml  # type: ignore
        from members.rafael.disparity.processing import generate_rectified  # type: ignore
        from members.rafael.disparity.utils import open_tiff_file  # type: ignore

        if os.path.exists(C.TEMP_PATH):
            shutil.rmtree(C.TEMP_PATH)
        os.makedirs(C.TEMP_PATH, exist_ok=False)
        self.close_log()
        self._log = open(os.path.join(C.TEMP_PATH, "log.txt"), "w")
        self.log("3D Point Cloud started")
        self.log(f"loading images from: {C.WV3_PATH}\n")
        selector = PairSelector(C.WV3_PATH)
        selector.discover_images()
        pairs = selector.select_pairs()
        for p in (C.TMP_STEREO_OUTPUT_PATH, C.TMP_CROPPED_IMAGES_PATH, C.TMP_DISPARITY_DEBUG_PATH):
            os.makedirs(p, exist_ok=False)
        self.log("preprocessing pairs")
        if is_debug_pair:
            a, b = C.PAIR_DECENT_RESULTS[0]
            pairs = [p for p in pairs if {p.img1.filename, p.img2.filename} == {a, b}]
        elif is_one_random_pair:
            pairs = [pairs[np.random.randint(0, min(n, len(pairs)))]]
        else:
            pairs = pairs[:n]
        for pair in pairs:
            for img in (pair.img1, pair.img2):
                name = img.filename + ".tif"
                if not os.path.exists(img.path):
                    self.log(f"image not found  {img.path}")
                    raise ImageNotFound(img.path)
                if os.path.exists(os.path.join(C.TMP_CROPPED_IMAGES_PATH, name)):
                    continue
                try:
                    area = get_crop_area_from_kml(img, str(kml_path))
                    self.log(f"crop area for {img.filename}: {area}")
                    generate_cropped(img, C.TMP_CROPPED_IMAGES_PATH, name, area)
                    self.log(f"generated cropped image for {img.filename} at {C.TMP_CROPPED_IMAGES_PATH}")
                except Exception as e:   # noqa: BLE001 -- plugin.py:89-91
                    self.log(f"error: Cropping failed for {img.filename}: {str(e)}")
                    raise CropFailed(str(e)) from e
        for pair_id, pair in enumerate(pairs):
            self.log("ASP stereo rectification...")
            out_path = generate_rectified(pair, pair_id, C.TMP_STEREO_OUTPUT_PATH)
            self.log(f"Rectification complete, output: {out_path}")
            self.log("Generating disparity map...")
            gathers = use_gpu_gathers(dmod) if self.gpu_gathers else contextlib.nullcontext()
            with gathers:
                disparity, validity, photo = dmod.disparity_map(pair, pair_id, C.TMP_STEREO_OUTPUT_PATH,
                                                                C.TMP_CROPPED_IMAGES_PATH, C.TMP_DISPARITY_DEBUG_PATH)
            self.log("Disparity map generated successfully")
            image_layers = []
            if is_debug_mode:   # plugin.py:120-145
                self.log("Loading  basic cropped image for display...")
                # the cropped inputs are opened unconditionally (plugin.py:123, 128): a missing
                # crop raises and becomes the reference's "Error: ..." layer; the rectified
                # images only when present (plugin.py:134, 141)
                sources = [(os.path.join(C.TMP_CROPPED_IMAGES_PATH, pair.img1.cropped_name), "Input Left", True),
                           (os.path.join(C.TMP_CROPPED_IMAGES_PATH, pair.img2.cropped_name), "Input Right", True),
                           (os.path.join(C.TMP_STEREO_OUTPUT_PATH, str(pair_id), "results", "out-L.tif"),
                            "Rectified Left", False),
                           (os.path.join(C.TMP_STEREO_OUTPUT_PATH, str(pair_id), "results", "out-R.tif"),
                            "Rectified Right", False)]
                for path, label, required in sources:
                    if required or os.path.exists(path):
                        im = open_tiff_file(path)
                        image_layers.append((normalise_for_display(im, im > 0),
                                             {"name": f"{PREFIX} {label}", "colormap": "gray"}, "image"))
            yield PairProducts(disparity=disparity, validity=np.asarray(validity, dtype=bool),
                               photoconsistency=photo, image_layers=image_layers)
