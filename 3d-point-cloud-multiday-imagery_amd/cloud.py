"""Per-pair point-cloud assembly on the GPU.

``assemble_cloud`` is the float64 block of ``members/rafael/disparity/plugin.py:147-192``
(height map from the SGBM/WLS disparity, validity mask, row-major compaction,
plane fit oriented to +z, relative height, 2/98-percentile ``height`` property,
``points_coords = stack([z, y, x])``) done by the HIP kernels of
``csrc/pcm_cloud.hpp`` through ``pcm_cloud_assemble``.  No CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .engine import _ptr, _stream

MAX_DISP = 288   # members/rafael/disparity/constants.py:54-57


def assemble_cloud(disparity, validity=None, max_disp: int = MAX_DISP):
    """Returns (points (M,3) float64 z,y,x, h_norm (M,) float64, normal (3,)) as host arrays."""
    pts, hn, normal = assemble_cloud_device(disparity, validity, max_disp)
    return pts.cpu().numpy(), hn.cpu().numpy(), normal


def assemble_cloud_device(disparity, validity=None, max_disp: int = MAX_DISP):
    """As ``assemble_cloud`` but the points and h_norm stay on the device (views of
    the kernels' outputs): the plugin feeds them to the fused K-means directly."""
    if not torch.cuda.is_available():
        raise _lib.PcmError("assemble_cloud needs a HIP device (no CPU fallback)")
    d = torch.as_tensor(np.asarray(disparity) if not isinstance(disparity, torch.Tensor) else disparity)
    d = d.to("cuda", torch.float64).contiguous()
    if d.dim() != 2:
        raise ValueError("disparity must be (H, W)")
    H, W = d.shape
    v = None
    if validity is not None:
        v = torch.as_tensor(np.asarray(validity, dtype=np.uint8) if not isinstance(validity, torch.Tensor)
                            else validity).to("cuda", torch.uint8).contiguous()
        if tuple(v.shape) != (H, W):
            raise ValueError("validity must match the disparity shape")
    pts = torch.empty((H * W, 3), dtype=torch.float64, device="cuda")
    hn = torch.empty(H * W, dtype=torch.float64, device="cuda")
    m = ctypes.c_int64(0)
    normal = np.zeros(3, np.float64)
    lib = _lib.load()
    _lib.check(lib.pcm_cloud_assemble(_ptr(d), _ptr(v) if v is not None else None, H, W, float(max_disp / 2),
                                      _ptr(pts), _ptr(hn), ctypes.byref(m), normal.ctypes.data_as(ctypes.c_void_p),
                                      _stream()), "pcm_cloud_assemble")
    M = int(m.value)
    if M < 3:
        # the reference's plane fit takes ``Vh[2]`` of the thin SVD of the (M, 3)
        # centred points (plugin.py:164-165), which has min(M, 3) rows: fewer than
        # 3 valid pixels raise numpy's IndexError there, and the run becomes one
        # "Error: <msg>" layer (plugin.py:236-241) -- same exception, same text
        raise IndexError(f"index 2 is out of bounds for axis 0 with size {M}")
    return pts[:M], hn[:M], normal
