"""MI355X-native multi-day point-cloud K-means (Lloyd) reconstruction step.

Drop-in for the K-means step of the ``members/rafael`` "Multi-day 3D Point
Cloud" plugin (see DESIGN.md / INTEGRATION.md).  Import name: ``pcm_amd``
(the repository-root shim ``pcm_amd.py`` maps it onto this directory).

Public API
----------
lloyd_fit(X, centers_init, max_iter, tol, group=None)  -> LloydResult
kmeans_plusplus(X, n_clusters, random_state=...)       -> (centers, indices), GPU k-means++
assemble_cloud(disparity, validity, max_disp=288)      -> per-pair (z,y,x) cloud + height property (GPU)
KMeans(n_clusters, init, n_init, ...).fit_predict(X)   -> the reference's KMeans call site (core.py:227-228)
dense_fit / dense_kmeanspp                             -> generic-D (float32/float64) Lloyd + k-means++ (GPU)
photoconsistency_map / left_right_consistency          -> stereo consistency gathers (GPU, processing.py / disparity.py)
kmeans_fuse(clouds, n_clusters, ...)                   -> napari layer tuples
HeightMapExtractor                                     -> SatellitePlugin drop-in
Engine                                                 -> the C-ABI engine wrapper
"""
from .fixed import QBITS, fixed_q  # noqa: F401
from .lloyd import LloydResult, lloyd_fit  # noqa: F401

__all__ = ["lloyd_fit", "LloydResult", "fixed_q", "QBITS", "Engine", "kmeans_fuse", "HeightMapExtractor",
           "build_library", "kmeans_plusplus", "assemble_cloud", "KMeans", "dense_fit", "dense_kmeanspp",
           "photoconsistency_map", "left_right_consistency"]


def __getattr__(name):
    # lazy: the engine needs torch + the HIP library, the plugin needs neither at import
    if name == "Engine":
        from .engine import Engine
        return Engine
    if name in ("kmeans_fuse", "HeightMapExtractor", "PREFIX"):
        from . import plugin
        return getattr(plugin, name)
    if name == "KMeans":
        from .estimator import KMeans
        return KMeans
    if name == "assemble_cloud":
        from .cloud import assemble_cloud
        return assemble_cloud
    if name in ("dense_fit", "dense_kmeanspp"):
        from . import dense
        return getattr(dense, name)
    if name in ("photoconsistency_map", "left_right_consistency"):
        from . import stereo
        return getattr(stereo, name)
    if name == "kmeans_plusplus":
        from .kpp import kmeans_plusplus
        return kmeans_plusplus
    if name == "build_library":
        from ._lib import build
        return build
    raise AttributeError(name)
