"""CPU restatement of the per-pair cloud assembly of the reference plugin.

TEST INFRASTRUCTURE ONLY (same rules as ``oracle/lloyd_ref.py``).

Restates ``members/rafael/disparity/plugin.py:147-192`` literally, in float64:

* ``height_map = -disparity / 16`` (:148); valid = finite & ``|h| <= MAX_DISP/2``
  & validity (:151-152, ``MAX_DISP = 288`` from constants.py:54-57);
* ``y, x = np.where(valid)``; ``P = stack([x, y, z])`` (:157-160);
* plane fit: mean, SVD of the centred points, ``normal = Vh[2]`` oriented to +z
  (:161-168); relative height ``P_c . normal`` (:171);
* ``h_min, h_max`` = 2nd / 98th percentiles (linear), ``h_norm`` clipped to
  [0, 1] (:181-187); ``z -= h_min``; ``points = stack([z, y, x])`` (:192).

The GPU path (``csrc/pcm_cloud.hpp``) computes the plane from the 3x3
covariance (the right singular vectors of ``P_c`` are its eigenvectors) and
sums in a different order, so parity is to float64 rounding (tests: 1e-9
relative), not bit-exact.
"""
from __future__ import annotations

import numpy as np

MAX_DISP = 288


def assemble(disparity: np.ndarray, validity: np.ndarray | None = None, max_disp: int = MAX_DISP):
    """Returns (points (M,3) float64 in z,y,x order, h_norm (M,), normal (3,))."""
    height_map = -np.asarray(disparity).astype(float) / 16.0
    limit = max_disp / 2
    valid = np.isfinite(height_map) & (np.abs(height_map) <= limit)
    if validity is not None:
        valid &= np.asarray(validity, dtype=bool)
    y, x = np.where(valid)
    z = height_map[valid]
    P = np.stack([x, y, z], axis=1)
    center = np.mean(P, axis=0)
    Pc = P - center
    _, _, Vh = np.linalg.svd(Pc, full_matrices=False)
    normal = Vh[2]
    if np.dot(normal, np.array([0, 0, 1])) < 0:
        normal = -normal
    z = np.dot(Pc, normal)
    h_min = np.percentile(z, 2)
    h_max = np.percentile(z, 98)
    h_norm = np.clip((z - h_min) / (h_max - h_min + 1e-6), 0, 1)
    z = z - h_min
    return np.stack([z, y, x], axis=1), h_norm, normal
