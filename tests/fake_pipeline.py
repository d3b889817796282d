"""Synthetic stand-in for the reference's per-pair stereo pipeline (TEST ONLY).

The reference's HeightMapExtractor.run (members/rafael/disparity/plugin.py:36-243)
needs GDAL, OpenCV, rasterio and the NASA Ames Stereo Pipeline, none of which
exist here.  This produces layers of the same shape for each synthetic "pair":
a height map from a smooth synthetic disparity, the valid mask, the point
cloud assembly of plugin.py:147-192 restated in numpy (P = [x, y, z] of valid
pixels, SVD plane fit with the normal oriented to +z, relative height,
2/98-percentile height property, z shifted by its 2nd percentile,
points_coords = stack([z, y, x])) and the points layer params of
plugin.py:220-233.
"""
import numpy as np

PREFIX = "[Multi-day 3D Point Cloud]"


def pair_cloud(height_map, valid):
    y, x = np.where(valid)
    z = height_map[valid]
    P = np.stack([x, y, z], axis=1).astype(np.float64)
    center = P.mean(axis=0)
    Pc = P - center
    _, _, Vh = np.linalg.svd(Pc, full_matrices=False)
    normal = Vh[2]
    if np.dot(normal, [0, 0, 1]) < 0:
        normal = -normal
    z = Pc @ normal
    h_min, h_max = np.percentile(z, 2), np.percentile(z, 98)
    h_norm = np.clip((z - h_min) / (h_max - h_min + 1e-6), 0, 1)
    z = z - h_min
    return np.stack([z, y, x], axis=1), h_norm


class SyntheticPairExtractor:
    """Object with the reference extractor's run() signature."""

    def __init__(self, n_pairs=2, shape=(120, 160), seed=0, fail=False):
        self.n_pairs, self.shape, self.seed, self.fail = n_pairs, shape, seed, fail

    def run(self, kml_path, is_debug_mode=True, is_debug_pair=False, is_one_random_pair=True, n=10):
        if self.fail:
            return [(np.ones((100, 100)), {"name": "Error: synthetic failure"}, "image")]
        rng = np.random.default_rng(self.seed)
        H, W = self.shape
        yy, xx = np.mgrid[0:H, 0:W]
        layers = []
        for p in range(min(self.n_pairs, n)):
            disparity = -16.0 * (8 * np.sin(xx / 23.0 + p) + 5 * np.cos(yy / 17.0) + rng.normal(0, 0.3, (H, W)))
            height_map = -disparity / 16.0                         # plugin.py:148
            valid = np.isfinite(height_map) & (np.abs(height_map) <= 144) & (rng.random((H, W)) > 0.1)
            coords, h_norm = pair_cloud(height_map, valid)
            layers.append((height_map, {"name": f"{PREFIX} Disparity", "colormap": "turbo"}, "image"))
            layers.append((coords, {"name": f"{PREFIX} 3D Point Cloud", "size": 2,
                                    "properties": {"height": h_norm}, "scale": (1, 1, 1), "opacity": 0.8,
                                    "face_colormap": "turbo", "face_color": "height"}, "points"))
        return layers


class SyntheticStages:
    """Stand-in for pcm_amd.pipeline.ReferenceStereoStages: per-pair products
    (disparity, validity mask, photoconsistency, debug image layers) of the
    shape the reference's disparity_map returns (disparity.py:21-226)."""

    def __init__(self, n_pairs=2, shape=(120, 160), seed=0, fail_at=None, fail=None, n_valid=None, dark_at=None):
        self.n_pairs, self.shape, self.seed, self.fail_at, self.fail = n_pairs, shape, seed, fail_at, fail
        # n_valid = (pair, m): that pair keeps only its first m valid pixels (row-major);
        # dark_at = pair whose photoconsistency is nowhere positive
        self.n_valid, self.dark_at = n_valid, dark_at
        self.logged = []

    def log(self, msg):
        self.logged.append(msg)

    def pairs(self, kml_path, is_debug_mode=True, is_debug_pair=False, is_one_random_pair=True, n=10):
        from pcm_amd.pipeline import CropFailed, ImageNotFound, PairProducts
        if self.fail == "image":
            raise ImageNotFound("/data/WV3/PAN/missing.NTF")
        if self.fail == "crop":
            raise CropFailed("KML region outside the image")
        rng = np.random.default_rng(self.seed)
        H, W = self.shape
        yy, xx = np.mgrid[0:H, 0:W]
        for p in range(min(self.n_pairs, n)):
            if self.fail_at == p:
                raise RuntimeError("synthetic stereo failure")
            disparity = -16.0 * (8 * np.sin(xx / 23.0 + p) + 5 * np.cos(yy / 17.0) + rng.normal(0, 0.3, (H, W)))
            disparity[rng.random((H, W)) < 0.02] = 16.0 * 1000           # WLS sentinel
            validity = rng.random((H, W)) > 0.1
            photo = np.where(rng.random((H, W)) < 0.8, rng.uniform(0, 0.3, (H, W)), 0.0)
            if self.n_valid is not None and self.n_valid[0] == p:
                validity = np.zeros((H, W), bool)
                validity.flat[:self.n_valid[1]] = True
                disparity.flat[:self.n_valid[1]] = -16.0 * (1.0 + np.arange(self.n_valid[1]))   # in range
            if self.dark_at == p:
                photo = np.zeros((H, W))
            image_layers = [(rng.random((H, W)), {"name": f"{PREFIX} Input Left", "colormap": "gray"}, "image")] \
                if is_debug_mode else []
            yield PairProducts(disparity=disparity, validity=validity, photoconsistency=photo,
                               image_layers=image_layers)
