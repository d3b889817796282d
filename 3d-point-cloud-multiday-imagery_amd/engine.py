"""Thin torch-side wrapper of the C-ABI engine (``include/pcm_kmeans.h``).

Points, centres, labels and statistics are torch tensors on the engine's
device; every call passes ``tensor.data_ptr()`` and the current torch stream.
PyTorch is plumbing here (device memory, streams, torch.distributed); all the
arithmetic happens in the HIP kernels of ``csrc/``.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib

PCM_F32, PCM_F16 = 0, 1
RELOC_RECORD_BYTES = 32


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t: torch.Tensor):
    return ctypes.c_void_p(t.data_ptr())


class Engine:
    """One Lloyd engine on the current CUDA(HIP) device.

    Mirrors one ``_kmeans_single_lloyd`` run (sklearn/cluster/_kmeans.py:623-752)
    over this process's shard of the cloud.
    """

    def __init__(self, d: int, k: int, dtype=torch.float32, max_iter: int = 300):
        if not torch.cuda.is_available():
            raise _lib.PcmError("no HIP device visible: the Lloyd engine has no CPU fallback")
        self.lib = _lib.load()
        self.d, self.k, self.max_iter_cap = int(d), int(k), int(max_iter)
        if dtype not in (torch.float32, torch.float16):
            raise ValueError("points dtype must be float32 or float16")
        self.dtype = dtype
        self.device = torch.device("cuda", torch.cuda.current_device())
        self.stats_device = self.device
        h = ctypes.c_void_p()
        _lib.check(self.lib.pcm_engine_create(self.device.index, self.d, self.k,
                                              PCM_F16 if dtype == torch.float16 else PCM_F32,
                                              self.max_iter_cap, ctypes.byref(h)), "pcm_engine_create")
        self.h = h
        self.n = 0
        self.stats = None

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.pcm_engine_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ layout
    def bbox(self, X: torch.Tensor):
        X = self._check_points(X)
        lo = np.zeros(self.d)
        hi = np.zeros(self.d)
        mx = np.zeros(self.d)
        dp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        _lib.check(self.lib.pcm_layout_bbox(self.h, _ptr(X) if X.numel() else None, X.shape[0], _stream(),
                                            dp(lo), dp(hi), dp(mx)), "pcm_layout_bbox")
        self.n = X.shape[0]
        return lo, hi, mx

    def build(self, X: torch.Tensor, q, gidx0: int = 0):
        X = self._check_points(X)
        qa = np.ascontiguousarray(np.asarray(q, dtype=np.int32))
        _lib.check(self.lib.pcm_layout_build(self.h, _ptr(X) if X.numel() else None,
                                             qa.ctypes.data_as(ctypes.c_void_p), int(gidx0), _stream()),
                   "pcm_layout_build")
        cnt = ctypes.c_int64()
        p = ctypes.c_void_p()
        self.lib.pcm_stats_ptr(self.h, ctypes.byref(p), ctypes.byref(cnt))
        # statistics live in a torch tensor so torch.distributed can all-reduce them
        self.stats = torch.zeros(cnt.value, dtype=torch.int64, device=self.device)
        _lib.check(self.lib.pcm_bind_stats(self.h, _ptr(self.stats)), "pcm_bind_stats")

    def _check_points(self, X: torch.Tensor) -> torch.Tensor:
        if X.dim() != 2 or X.shape[1] != self.d:
            raise ValueError(f"points must be (N, {self.d})")
        if X.dtype != self.dtype:
            raise ValueError(f"points dtype {X.dtype} != engine dtype {self.dtype}")
        if X.device != self.device:
            raise ValueError("points must live on the engine's device")
        return X.contiguous()

    # ------------------------------------------------------------ fit
    def begin(self, C0: torch.Tensor, tol: float, max_iter: int):
        C0 = C0.to(device=self.device, dtype=torch.float32).contiguous()
        if tuple(C0.shape) != (self.k, self.d):
            raise ValueError(f"centres must be ({self.k}, {self.d})")
        self._c0 = C0
        _lib.check(self.lib.pcm_fit_begin(self.h, _ptr(C0), float(tol), int(max_iter), _stream()), "pcm_fit_begin")

    def iter_local(self):
        _lib.check(self.lib.pcm_iter_local(self.h, _stream()), "pcm_iter_local")

    def iter_global(self):
        _lib.check(self.lib.pcm_iter_global(self.h, _stream()), "pcm_iter_global")

    def iterate(self, n: int):
        _lib.check(self.lib.pcm_iterate(self.h, int(n), _stream()), "pcm_iterate")

    def status(self) -> dict:
        st = _lib.PcmStatus()
        _lib.check(self.lib.pcm_read_status(self.h, ctypes.byref(st), _stream()), "pcm_read_status")
        return dict(halt=st.halt, done=st.done, iter=st.iter, n_empty=st.n_empty, inertia=st.inertia,
                    last_changed=st.last_changed, last_shift=st.last_shift,
                    inertia_limbs=[int(v) for v in st.inertia_limbs], inertia_scale=int(st.inertia_scale),
                    inertia_overflow=int(st.inertia_overflow), list_rebuilds=int(st.list_rebuilds))

    def reloc_candidates(self, m: int) -> torch.Tensor:
        rec = torch.zeros(m * RELOC_RECORD_BYTES, dtype=torch.uint8, device=self.device)
        _lib.check(self.lib.pcm_reloc_candidates(self.h, int(m), _ptr(rec), _stream()), "pcm_reloc_candidates")
        return rec

    def reloc_apply(self, records: torch.Tensor):
        n_rec = records.numel() // RELOC_RECORD_BYTES
        _lib.check(self.lib.pcm_reloc_apply(self.h, _ptr(records), int(n_rec), _stream()), "pcm_reloc_apply")

    def final(self):
        _lib.check(self.lib.pcm_final(self.h, _stream()), "pcm_final")

    def labels(self) -> torch.Tensor:
        out = torch.empty(self.n, dtype=torch.int32, device=self.device)
        _lib.check(self.lib.pcm_labels(self.h, _ptr(out) if self.n else None, _stream()), "pcm_labels")
        return out

    def centers(self) -> torch.Tensor:
        out = torch.empty((self.k, self.d), dtype=torch.float32, device=self.device)
        _lib.check(self.lib.pcm_get_centers(self.h, _ptr(out), _stream()), "pcm_get_centers")
        return out

    def history(self, n: int):
        ch = np.zeros(self.max_iter_cap, dtype=np.uint64)
        sh = np.zeros(self.max_iter_cap, dtype=np.float64)
        _lib.check(self.lib.pcm_history(self.h, ch.ctypes.data_as(ctypes.c_void_p),
                                        sh.ctypes.data_as(ctypes.c_void_p), self.max_iter_cap, _stream()),
                   "pcm_history")
        return ch[:n].astype(np.int64), sh[:n]

    def timing(self, enable: bool):
        _lib.check(self.lib.pcm_timing(self.h, int(bool(enable))), "pcm_timing")

    def timing_read(self) -> dict:
        ms = np.zeros(3)
        cnt = ctypes.c_int()
        _lib.check(self.lib.pcm_timing_read(self.h, ms.ctypes.data_as(ctypes.c_void_p), ctypes.byref(cnt)),
                   "pcm_timing_read")
        return dict(assign_ms=ms[0], candidates_ms=ms[1], tail_ms=ms[2], iterations=cnt.value)

    def layout_info(self) -> dict:
        nc, nt = ctypes.c_int64(), ctypes.c_int64()
        g = (ctypes.c_int * 4)()
        _lib.check(self.lib.pcm_layout_info(self.h, ctypes.byref(nc), ctypes.byref(nt), g), "pcm_layout_info")
        return dict(ncells=nc.value, ntiles=nt.value, grid=list(g)[: self.d])

    def candidate_stats(self) -> dict:
        mean, mx, full = ctypes.c_double(), ctypes.c_int(), ctypes.c_int64()
        _lib.check(self.lib.pcm_candidate_stats(self.h, ctypes.byref(mean), ctypes.byref(mx), ctypes.byref(full),
                                                _stream()), "pcm_candidate_stats")
        return dict(mean=mean.value, max=mx.value, full_cells=full.value)


def synth_uniform(n: int, d: int, seed: int, start: int = 0, device=None) -> torch.Tensor:
    """Device-generated counter-based U[0,1) cloud (bit-identical to the CPU generator)."""
    lib = _lib.load()
    out = torch.empty((n, d), dtype=torch.float32, device=device or "cuda")
    _lib.check(lib.pcm_synth_uniform(_ptr(out) if n else None, int(n), int(d), ctypes.c_uint64(seed), int(start),
                                     _stream()), "pcm_synth_uniform")
    return out


def synth_rows(rows, d: int, seed: int, device=None) -> torch.Tensor:
    """Selected rows of the synthetic cloud (e.g. the initial centres)."""
    lib = _lib.load()
    r = torch.as_tensor(np.asarray(rows, dtype=np.int64), device=device or "cuda")
    out = torch.empty((r.numel(), d), dtype=torch.float32, device=r.device)
    _lib.check(lib.pcm_synth_rows(_ptr(out), _ptr(r), r.numel(), int(d), ctypes.c_uint64(seed), _stream()),
               "pcm_synth_rows")
    return out


def assign_bruteforce(X: torch.Tensor, C: torch.Tensor, q, stats: torch.Tensor = None):
    """Stateless brute-force E-step (+ optional statistics) over all K centres."""
    lib = _lib.load()
    X = X.contiguous()
    C = C.to(torch.float32).contiguous()
    n, d = X.shape
    labels = torch.empty(n, dtype=torch.int32, device=X.device)
    qa = np.ascontiguousarray(np.asarray(q, dtype=np.int32))
    _lib.check(lib.pcm_assign_bruteforce(_ptr(X), n, d, _ptr(C), C.shape[0], qa.ctypes.data_as(ctypes.c_void_p),
                                         _ptr(labels), _ptr(stats) if stats is not None else None, _stream()),
               "pcm_assign_bruteforce")
    return labels
