"""Drop-in "Multi-day 3D Point Cloud" plugin with the GPU K-means fusion step.

Boundary: the reference's ``HeightMapExtractor``
(members/rafael/disparity/plugin.py:22-243) builds one point cloud per stereo
pair -- ``points_coords = stack([z, y, x])`` (plugin.py:191-192) emitted as a
napari points layer (plugin.py:220-233) -- and never fuses days.  This class
keeps that component's public contract:

* ``name == "Multi-day 3D Point Cloud"`` (plugin.py:32-34; viewer.py:475-476
  dispatches the rafael tab on ``"3D Point Cloud" in plugin.name``);
* ``requires_image = False`` (plugin.py:29-30, read by viewer.py:107);
* ``run(kml_path, is_debug_mode=True, is_debug_pair=False,
  is_one_random_pair=True, n=10)`` (plugin.py:36-40, defaults from
  constants.py:5-10), called on a napari worker thread (widget.py:144-147);
* returns host numpy layers only, and never raises: failures come back as the
  reference's error image layers -- ``np.zeros((100, 100))`` named
  ``"error: image not found"`` / ``"error: <msg>"`` for a missing image or a
  failed crop (plugin.py:77-79, 89-91), otherwise ``np.ones((100, 100))`` named
  ``"Error: <msg>"`` (plugin.py:236-241); the stages write the run log
  ``TEMP/log.txt`` (plugin.py:49-50, 234, 240).

``run`` replays the reference's per-pair stereo stages (``pipeline.py``:
pair selection, crop, ASP rectification, SGBM/WLS disparity -- the reference's
own functions), assembles every pair's cloud ON THE GPU (``plugin.py:147-192``
-> ``cloud.assemble_cloud_device``), emits the reference's per-pair layers
(``plugin.py:176-233``) and appends the fused result of the K-means step that
slots in after plugin.py:192: a centroid points layer and the fused cloud with
a per-point ``cluster`` property.  The device clouds feed the K-means
(``pcm_amd.lloyd_fit``) without a host round trip.  ``base=`` keeps the older
mode: run an extractor with the reference's ``run`` and fuse the cloud layers
it returns.  Extra knobs (K, iterations, tolerance, export) are constructor
arguments so ``run``'s signature stays the reference's (viewer.py:118-127 would
turn extra ``run`` parameters into file pickers).
"""
from __future__ import annotations

import threading
from typing import Callable, List, Optional, Sequence

import numpy as np

try:  # inside the reference tree: the real plugin ABC
    from interface import SatellitePlugin  # type: ignore
except Exception:  # headless / tests
    from ._interface import SatellitePlugin

PREFIX = "[Multi-day 3D Point Cloud]"
CLOUD_LAYER_SUFFIX = "3D Point Cloud"
DEFAULTS = dict(is_debug_mode=True, is_debug_pair=False, is_one_random_pair=True, n=10)

_gpu_lock = threading.Lock()   # one fit at a time per process (widgets may run concurrently)


def _tolerance(X: np.ndarray, tol: float) -> float:
    """sklearn ``_tolerance`` (_kmeans.py:279-287): mean per-axis variance x tol."""
    if tol == 0 or X.shape[0] == 0:
        return 0.0
    return float(np.mean(np.var(X.astype(np.float64), axis=0)) * tol)


def _gpu_fit(X, C0: np.ndarray, max_iter: int, tol_abs: float):
    """X: host (N, 3) array, or the fused cloud already on the device."""
    import torch

    from .lloyd import LOCAL, lloyd_fit

    with _gpu_lock:
        Xt = X.to(torch.float32).contiguous() if isinstance(X, torch.Tensor) else \
            torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32)).cuda()
        Ct = torch.from_numpy(np.ascontiguousarray(C0, dtype=np.float32)).cuda()
        res = lloyd_fit(Xt, Ct, max_iter=max_iter, tol=tol_abs, group=LOCAL)   # whole cloud, this GPU
        torch.cuda.synchronize()
        return (res.labels.cpu().numpy(), res.centers.cpu().numpy(), float(res.inertia), int(res.n_iter))


def _norm(v: np.ndarray) -> np.ndarray:
    """Height property as the reference builds it: 2/98 percentiles -> [0, 1] (plugin.py:181-188)."""
    if v.size == 0:
        return v.astype(np.float64)
    lo, hi = np.percentile(v, 2), np.percentile(v, 98)
    return np.clip((v - lo) / (hi - lo + 1e-6), 0.0, 1.0)


def _gpu_kpp(X, k: int, seed: int) -> np.ndarray:
    import torch

    from .kpp import kmeans_plusplus

    with _gpu_lock:
        Xt = X.to(torch.float32).contiguous() if isinstance(X, torch.Tensor) else \
            torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32)).cuda()
        C, _ = kmeans_plusplus(Xt, k, random_state=seed)
        return C.cpu().numpy()


def export_fused(path, points: np.ndarray, result: dict):
    """On-disk fused cloud (row f4), the analogue of the reference's per-pair
    ``np.savez_compressed(path + 'consistency', ...)`` (disparity.py:220-224):
    fused (N, 3) z,y,x points (float64), per-point ``cluster`` labels, the (K, 3)
    centres, per-cluster counts, inertia and iterations.  ``load_fused`` reads it back."""
    np.savez_compressed(path, points=np.asarray(points, dtype=np.float64), cluster=result["labels"].astype(np.int32),
                        centers=np.asarray(result["centers"], dtype=np.float64),
                        counts=np.bincount(result["labels"], minlength=len(result["centers"])),
                        inertia=np.float64(result["inertia"]), n_iter=np.int64(result["n_iter"]))


def load_fused(path) -> dict:
    with np.load(path, allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def kmeans_fuse(clouds: Sequence[np.ndarray], n_clusters: int = 1024, max_iter: int = 300, tol: float = 1e-4,
                seed: int = 1, fit: Optional[Callable] = None, init: str = "rows", device_clouds=None,
                export_path=None):
    """Fuse per-pair (M_i, 3) z,y,x clouds into one K-means reconstruction.

    Returns (layers, result) where ``result`` has labels (N,), centers (K, 3),
    inertia, n_iter.  ``init``: ``"rows"`` = rows ``sorted(default_rng(seed).choice(N, K))``
    (SURVEY.md §8d); ``"k-means++"`` = GPU k-means++ with ``random_state=seed``
    (scikit-learn's KMeans default, sklearn/cluster/_kmeans.py:1012-1019).
    K is clipped to N.  ``device_clouds``: the same clouds already on the GPU
    (the plugin's GPU assembly) -- the K-means reads them there.  ``export_path``:
    also write the fused cloud (``export_fused``).
    """
    clouds = [np.asarray(c, dtype=np.float64).reshape(-1, 3) for c in clouds if np.asarray(c).size]
    if not clouds:
        raise ValueError("no point cloud layers to fuse")
    X = np.concatenate(clouds).astype(np.float32)          # boundary cast
    Xfit = X
    if device_clouds is not None and fit is None:
        import torch
        Xfit = torch.cat([c.reshape(-1, 3) for c in device_clouds if c.numel()]).to(torch.float32)   # same rounding
    n = X.shape[0]
    k = int(min(n_clusters, n))
    if init == "k-means++":
        C0 = _gpu_kpp(Xfit, k, seed)
    elif init == "rows":
        C0 = X[np.sort(np.random.default_rng(seed).choice(n, k, replace=False))]
    else:
        raise ValueError(f"init must be 'rows' or 'k-means++', got {init!r}")
    labels, centers, inertia, n_iter = (fit or _gpu_fit)(Xfit, C0, int(max_iter), _tolerance(X, tol))
    counts = np.bincount(labels, minlength=k)
    layers = [
        (centers.astype(np.float64),
         {"name": f"{PREFIX} Fused K-means Centroids", "size": 4,
          "properties": {"height": _norm(centers[:, 0].astype(np.float64)), "count": counts},
          "scale": (1, 1, 1), "opacity": 1.0, "face_colormap": "turbo", "face_color": "height"},
         "points"),
        (X.astype(np.float64),
         {"name": f"{PREFIX} Fused {CLOUD_LAYER_SUFFIX}", "size": 2,
          "properties": {"cluster": labels.astype(np.int32), "height": _norm(X[:, 0].astype(np.float64))},
          "scale": (1, 1, 1), "opacity": 0.8, "face_colormap": "turbo", "face_color": "cluster"},
         "points"),
    ]
    result = dict(labels=labels, centers=centers, inertia=inertia, n_iter=n_iter, n_points=n)
    if export_path is not None:
        export_fused(export_path, X.astype(np.float64), result)
    return layers, result


class HeightMapExtractor(SatellitePlugin):
    """Multi-day 3D point clouds from WV3 stereo pairs, fused by GPU K-means."""

    requires_image = False

    def __init__(self, base=None, n_clusters: int = 1024, max_iter: int = 300, tol: float = 1e-4,
                 fit: Optional[Callable] = None, init: str = "rows", seed: int = 1, stages=None,
                 export_path=None, _assemble: Optional[Callable] = None):
        self._base = base
        self._stages = stages
        self.export_path = export_path
        self._assemble = _assemble   # tests: a CPU stand-in for the GPU assembly (disparity, validity) -> (pts, h_norm)
        self.init = init
        self.seed = seed
        self.n_clusters = n_clusters
        self.max_iter = max_iter
        self.tol = tol
        self._fit = fit
        self.last_result = None

    @property
    def name(self):
        return "Multi-day 3D Point Cloud"

    def _gpu_stages_run(self, stages, kml_path, is_debug_mode, is_debug_pair, is_one_random_pair, n) -> List:
        from .pipeline import pair_layers
        layers, host_clouds, dev_clouds = [], [], []
        for pp in stages.pairs(kml_path, is_debug_mode=is_debug_mode, is_debug_pair=is_debug_pair,
                               is_one_random_pair=is_one_random_pair, n=n):
            layers += list(pp.image_layers)
            if self._assemble is not None:
                pts, hn = self._assemble(pp.disparity, pp.validity)
                dev = None
            else:
                from .cloud import assemble_cloud_device
                with _gpu_lock:
                    dev, hn_d, _ = assemble_cloud_device(pp.disparity, pp.validity)
                    pts, hn = dev.cpu().numpy(), hn_d.cpu().numpy()
            layers += pair_layers(pp, pts, hn)
            host_clouds.append(pts)
            dev_clouds.append(dev)
        if not host_clouds:
            return layers
        use_dev = self._fit is None and all(d is not None for d in dev_clouds)
        fused, self.last_result = kmeans_fuse(host_clouds, self.n_clusters, self.max_iter, self.tol, seed=self.seed,
                                              fit=self._fit, init=self.init,
                                              device_clouds=dev_clouds if use_dev else None,
                                              export_path=self.export_path)
        return layers + fused

    def _stages_run(self, kml_path, is_debug_mode, is_debug_pair, is_one_random_pair, n) -> List:
        from .pipeline import CropFailed, ImageNotFound, ReferenceStereoStages
        stages = self._stages or ReferenceStereoStages()
        log = getattr(stages, "log", lambda msg: None)
        try:
            layers = self._gpu_stages_run(stages, kml_path, is_debug_mode, is_debug_pair, is_one_random_pair, n)
            log(f"Added {len(layers)} layers to Napari")
            return layers
        except ImageNotFound:                      # plugin.py:77-79
            return [(np.zeros((100, 100)), {"name": "error: image not found"}, "image")]
        except CropFailed as e:                    # plugin.py:89-91
            return [(np.zeros((100, 100)), {"name": f"error: {str(e)}"}, "image")]
        except Exception as e:                     # plugin.py:236-241
            import traceback
            traceback.print_exc()
            log(f"Error: {str(e)}\n{traceback.format_exc()}")
            return [(np.ones((100, 100)), {"name": f"Error: {str(e)}"}, "image")]
        finally:
            getattr(stages, "close_log", lambda: None)()

    def run(self, kml_path, is_debug_mode: bool = DEFAULTS["is_debug_mode"],
            is_debug_pair: bool = DEFAULTS["is_debug_pair"],
            is_one_random_pair: bool = DEFAULTS["is_one_random_pair"], n: int = DEFAULTS["n"]) -> List:
        try:
            if self._base is None:
                return self._stages_run(kml_path, is_debug_mode, is_debug_pair, is_one_random_pair, n)
            layers = list(self._base.run(kml_path, is_debug_mode=is_debug_mode, is_debug_pair=is_debug_pair,
                                         is_one_random_pair=is_one_random_pair, n=n))
            clouds = [data for data, params, kind in layers
                      if kind == "points" and str(params.get("name", "")).endswith(CLOUD_LAYER_SUFFIX)]
            if not clouds:   # the pipeline returned only images (or an error layer): pass it through
                return layers
            fused, self.last_result = kmeans_fuse(clouds, self.n_clusters, self.max_iter, self.tol, seed=self.seed,
                                                  fit=self._fit, init=self.init, export_path=self.export_path)
            return layers + fused
        except Exception as e:   # reference convention: an error layer, never an exception
            import traceback
            traceback.print_exc()
            return [(np.ones((100, 100)), {"name": f"Error: {e}"}, "image")]
