"""CPU restatement of the stereo consistency gathers.

TEST INFRASTRUCTURE ONLY (same rules as ``oracle/lloyd_ref.py``): only
``tests/`` may import it, as the checker; the product path never does.

* ``photoconsistency_map`` -- ``members/rafael/disparity/processing.py:94-115``:
  for every pixel, ``xd = round(x - d)`` (NumPy rounds half to even); the pixel
  is undefined when ``d`` is NaN, ``xd`` falls outside ``[0, W)`` or
  ``d < min_disp``; defined pixels get ``|right[y, xd] - left[y, x]| / 255``
  (float64), undefined ones 0.
* ``left_right_consistency`` -- ``members/rafael/disparity/disparity.py:229-250``:
  same gather rule; defined pixels get ``|right_disp[y, xd] + left_disp[y, x]|``,
  undefined ones ``max_disp`` (default 80).  The caller thresholds it
  (``< 3``, ``disparity.py:170-172``).

Pinned: equal (bitwise) to the reference's own functions run on synthetic
inputs, ``tests/golden/stereo/consistency.npz`` (``tests/golden/make_stereo_golden.py``).
"""
from __future__ import annotations

import numpy as np


def _gather(disp: np.ndarray, min_disp: float):
    H, W = disp.shape
    ys, xs = np.mgrid[0:H, 0:W]
    with np.errstate(invalid="ignore"):
        xd_f = np.round(xs - disp)                   # half to even, NaN stays NaN
    undefined = np.isnan(disp) | ~(xd_f >= 0) | ~(xd_f < W) | (disp < min_disp)
    xd = np.where(undefined, xs, np.nan_to_num(xd_f, nan=0.0)).astype(np.int64)
    return ys, xs, xd, undefined


def photoconsistency_map(left, right, left_disp, min_disp):
    left_disp = np.asarray(left_disp, dtype=np.float64)
    ys, xs, xd, undefined = _gather(left_disp, min_disp)
    diff = np.abs(np.asarray(right)[ys, xd].astype(float) - np.asarray(left)[ys, xs].astype(float)) / 255.0
    diff[undefined] = 0
    return diff


def left_right_consistency(left_disp, right_disp, min_disp, max_disp=80):
    left_disp = np.asarray(left_disp, dtype=np.float64)
    right_disp = np.asarray(right_disp, dtype=np.float64)
    ys, xs, xd, undefined = _gather(left_disp, min_disp)
    diff = np.abs(right_disp[ys, xd] + left_disp[ys, xs])
    diff[undefined] = max_disp
    return diff
