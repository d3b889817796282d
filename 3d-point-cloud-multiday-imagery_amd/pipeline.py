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
* ``pair_layers(...)`` rebuilds the per-pair layers of ``plugin.py:176-233``
  from the GPU assembly (``cloud.assemble_cloud_device``) -- the height-map
  image (``normalise_for_display`` of the relative heights equals the
  assembly's ``h_norm`` at valid pixels), photoconsistency, invalid mask and
  the 3D point cloud layer -- while the device copy of each cloud feeds the
  fused K-means without a host round trip.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Iterator, List

import numpy as np

PREFIX = "[Multi-day 3D Point Cloud]"
MASK_COLORMAP = {"colors": [[0.0, 0.0, 0.0, 0.0], [0.0, 0.0, 0.0, 1.0]], "name": "mask_blackout",
                 "interpolation": "linear"}


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
    valid = pp.photoconsistency > 0            # plugin.py:194
    layers.append((normalise_for_display(pp.photoconsistency, valid) if valid.any() else
                   np.zeros((H, W)), {"name": f"{PREFIX} Photoconsistency", "colormap": "turbo", "scale": (1, 1)},
                   "image"))
    layers.append(((~valid).astype(np.float32), {"name": f"{PREFIX} Invalid Mask", "colormap": MASK_COLORMAP,
                                                   "scale": (1, 1), "contrast_limits": [0, 1]}, "image"))
    layers.append((points, {"name": f"{PREFIX} 3D Point Cloud", "size": 2, "properties": {"height": h_norm},
                            "scale": (1, 1, 1), "opacity": 0.8, "face_colormap": "turbo", "face_color": "height"},
                   "points"))
    return layers


class ReferenceStereoStages:
    """plugin.py:45-145 with the reference's functions (runs inside the reference tree)."""

    def pairs(self, kml_path, is_debug_mode: bool = True, is_debug_pair: bool = False,
              is_one_random_pair: bool = True, n: int = 10) -> Iterator[PairProducts]:
        import shutil

        from members.rafael.disparity import constants as C  # type: ignore
        from members.rafael.disparity.disparity import disparity_map  # type: ignore
        from members.rafael.disparity.pair_selector import PairSelector  # type: ignore
        from members.rafael.disparity.preprocessing import generate_cropped, get_crop_area_from_kml  # type: ignore
        from members.rafael.disparity.processing import generate_rectified  # type: ignore
        from members.rafael.disparity.utils import open_tiff_file  # type: ignore

        if os.path.exists(C.TEMP_PATH):
            shutil.rmtree(C.TEMP_PATH)
        os.makedirs(C.TEMP_PATH, exist_ok=False)
        selector = PairSelector(C.WV3_PATH)
        selector.discover_images()
        pairs = selector.select_pairs()
        for p in (C.TMP_STEREO_OUTPUT_PATH, C.TMP_CROPPED_IMAGES_PATH, C.TMP_DISPARITY_DEBUG_PATH):
            os.makedirs(p, exist_ok=False)
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
                    raise FileNotFoundError(f"image not found {img.path}")
                if not os.path.exists(os.path.join(C.TMP_CROPPED_IMAGES_PATH, name)):
                    generate_cropped(img, C.TMP_CROPPED_IMAGES_PATH, name, get_crop_area_from_kml(img, str(kml_path)))
        for pair_id, pair in enumerate(pairs):
            generate_rectified(pair, pair_id, C.TMP_STEREO_OUTPUT_PATH)
            disparity, validity, photo = disparity_map(pair, pair_id, C.TMP_STEREO_OUTPUT_PATH,
                                                       C.TMP_CROPPED_IMAGES_PATH, C.TMP_DISPARITY_DEBUG_PATH)
            image_layers = []
            if is_debug_mode:   # plugin.py:119-145
                sources = [(os.path.join(C.TMP_CROPPED_IMAGES_PATH, pair.img1.cropped_name), "Input Left"),
                           (os.path.join(C.TMP_CROPPED_IMAGES_PATH, pair.img2.cropped_name), "Input Right"),
                           (os.path.join(C.TMP_STEREO_OUTPUT_PATH, str(pair_id), "results", "out-L.tif"),
                            "Rectified Left"),
                           (os.path.join(C.TMP_STEREO_OUTPUT_PATH, str(pair_id), "results", "out-R.tif"),
                            "Rectified Right")]
                for path, label in sources:
                    if os.path.exists(path):
                        im = open_tiff_file(path)
                        image_layers.append((normalise_for_display(im, im > 0),
                                             {"name": f"{PREFIX} {label}", "colormap": "gray"}, "image"))
            yield PairProducts(disparity=disparity, validity=np.asarray(validity, dtype=bool),
                               photoconsistency=photo, image_layers=image_layers)
