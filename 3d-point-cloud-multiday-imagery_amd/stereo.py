"""Stereo consistency gathers on the GPU.

Drop-ins for the reference's per-pixel NumPy gathers, with the same names,
arguments and results:

* ``photoconsistency_map(left, right, left_disp, min_disp)`` --
  ``members/rafael/disparity/processing.py:94-115``;
* ``left_right_consistency(left_disp, right_disp, min_disp, max_disp=80)`` --
  ``members/rafael/disparity/disparity.py:229-250``; ``threshold=`` also returns
  the ``< threshold`` mask (``disparity.py:170-172``) from the same pass.

NumPy arrays in -> NumPy arrays out (uploaded, computed by the HIP kernels of
``csrc/pcm_stereo.hip``, copied back); HIP device tensors in -> device tensors
out, stream-ordered.  There is no CPU fallback.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .engine import _ptr, _stream

PCM_F32, PCM_F64 = 0, 2


def _dev(a, dtype=None):
    if isinstance(a, torch.Tensor):
        if not a.is_cuda:
            raise _lib.PcmError("stereo gathers expect HIP device tensors or NumPy arrays")
        t = a
    else:
        t = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    return t.contiguous()


def _img(a):
    t = _dev(a)
    if t.dtype not in (torch.float32, torch.float64):
        t = t.to(torch.float64)   # reference: .astype(float)
    return t


def photoconsistency_map(left, right, left_disp, min_disp):
    host = not isinstance(left_disp, torch.Tensor)
    d = _dev(left_disp, torch.float64)
    if d.dim() != 2:
        raise ValueError("left_disp must be (H, W)")
    H, W = d.shape
    L, R = _img(left), _img(right)
    if L.dtype != R.dtype:
        L, R = L.to(torch.float64), R.to(torch.float64)
    if tuple(L.shape) != (H, W) or tuple(R.shape) != (H, W):
        raise ValueError("left, right and left_disp must have the same (H, W) shape")
    out = torch.empty((H, W), dtype=torch.float64, device=d.device)
    _lib.check(_lib.load().pcm_photoconsistency(_ptr(L), _ptr(R), PCM_F32 if L.dtype == torch.float32 else PCM_F64,
                                                _ptr(d), H, W, float(min_disp), _ptr(out), _stream()),
               "pcm_photoconsistency")
    return out.cpu().numpy() if host else out


def left_right_consistency(left_disp, right_disp, min_disp, max_disp=80, threshold=None):
    host = not isinstance(left_disp, torch.Tensor)
    ld, rd = _dev(left_disp, torch.float64), _dev(right_disp, torch.float64)
    if ld.dim() != 2 or ld.shape != rd.shape:
        raise ValueError("left_disp and right_disp must be (H, W) of one shape")
    H, W = ld.shape
    out = torch.empty((H, W), dtype=torch.float64, device=ld.device)
    below = torch.empty((H, W), dtype=torch.uint8, device=ld.device) if threshold is not None else None
    _lib.check(_lib.load().pcm_lr_consistency(_ptr(ld), _ptr(rd), H, W, float(min_disp), float(max_disp), _ptr(out),
                                              _ptr(below) if below is not None else None,
                                              float(threshold) if threshold is not None else 0.0, _stream()),
               "pcm_lr_consistency")
    if threshold is None:
        return out.cpu().numpy() if host else out
    below = below.bool()
    return (out.cpu().numpy(), below.cpu().numpy()) if host else (out, below)
