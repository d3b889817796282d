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
# one engine holds fewer than 2^28 - 16 padded points (pcm_engine.hip, pcm_layout_build's check);
# larger clouds are sharded over engines / ranks
ENGINE_MAX_POINTS = (1 << 28) - 4096


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
        # statistics live in a torch tensor so torch.distributed can all-reduce them;
        # allocated (and torch's fill kernel loaded) here, at engine creation, not in
        # the first layout (pcm_fit_begin zeroes them for every fit)
        cnt = ctypes.c_int64()
        p = ctypes.c_void_p()
        _lib.check(self.lib.pcm_stats_ptr(self.h, ctypes.byref(p), ctypes.byref(cnt)), "pcm_stats_ptr")
        self.stats = torch.zeros(cnt.value, dtype=torch.int64, device=self.device)
        _lib.check(self.lib.pcm_bind_stats(self.h, _ptr(self.stats)), "pcm_bind_stats")

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.pcm_engine_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reserve(self, n: int):
        """Grow the point-sized device buffers for layouts of up to ``n`` points
        now (``pcm_engine_reserve``): a fresh process's first large allocations
        map and clear new VRAM, which would otherwise land in the first layout."""
        _lib.check(self.lib.pcm_engine_reserve(self.h, int(n), _stream()), "pcm_engine_reserve")

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

    def set_shard(self, rows: torch.Tensor, n_global: int):
        """This engine's cloud is a spatial shard (``pcm_layout_shard``): global
        row of every local point (relocation tie-break), points on all ranks."""
        rows = rows.to(device=self.device, dtype=torch.int32).contiguous()
        if rows.numel() != self.n:
            raise ValueError("one global row per local point")
        _lib.check(self.lib.pcm_layout_shard(self.h, _ptr(rows) if rows.numel() else None, int(n_global), _stream()),
                   "pcm_layout_shard")

    # spatial slab sharding (stateless operators, csrc/pcm_shard.hip)
    def shard_hist(self, X, axis, lo, inv, nbins):
        return shard_hist(X, axis, lo, inv, nbins)

    def shard_partition(self, X, axis, lo, inv, nbins, owner, world, gidx0):
        return shard_partition(X, axis, lo, inv, nbins, owner, world, gidx0)

    def shard_scatter_labels(self, labels, rows, gidx0, n):
        return shard_scatter_labels(labels, rows, gidx0, n)

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

    def exchange(self, x, phase: int = 3):
        """The statistics summed over the ranks by the peer exchange ``x``
        (``pcm_iter_exchange``; xchg.PeerExchange), in place of the all-reduce."""
        _lib.check(self.lib.pcm_iter_exchange(self.h, x.h, int(phase), _stream()), "pcm_iter_exchange")

    def iterate(self, n: int):
        _lib.check(self.lib.pcm_iterate(self.h, int(n), _stream()), "pcm_iterate")

    def status_post(self):
        """Queue a status snapshot behind the work enqueued so far (no drain)."""
        _lib.check(self.lib.pcm_status_post(self.h, _stream()), "pcm_status_post")

    def status_wait(self) -> dict:
        """The snapshot of the last ``status_post``, once it has landed."""
        st = _lib.PcmStatus()
        _lib.check(self.lib.pcm_status_wait(self.h, ctypes.byref(st)), "pcm_status_wait")
        return self._status_dict(st)

    def status(self) -> dict:
        st = _lib.PcmStatus()
        _lib.check(self.lib.pcm_read_status(self.h, ctypes.byref(st), _stream()), "pcm_read_status")
        return self._status_dict(st)

    @staticmethod
    def _status_dict(st) -> dict:
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

    def time_assign(self, reps: int) -> float:
        """Mean ms of `reps` back-to-back assign launches (calibration; the fit must begin again)."""
        ms = ctypes.c_double()
        _lib.check(self.lib.pcm_time_assign(self.h, int(reps), _stream(), ctypes.byref(ms)), "pcm_time_assign")
        return ms.value

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

    def stream_bytes(self) -> dict:
        """Bytes the assign kernel streams per iteration (compressed tiles at 8 B/pt)."""
        b, z = ctypes.c_double(), ctypes.c_int64()
        _lib.check(self.lib.pcm_layout_stream_bytes(self.h, ctypes.byref(b), ctypes.byref(z)), "pcm_layout_stream_bytes")
        return dict(bytes=b.value, compressed_points=z.value)

    def assign_kernel(self) -> str:
        buf = ctypes.create_string_buffer(128)
        _lib.check(self.lib.pcm_assign_kernel_name(self.h, buf, 128), "pcm_assign_kernel_name")
        return buf.value.decode()

    def candidate_stats(self) -> dict:
        mean, mx, full = ctypes.c_double(), ctypes.c_int(), ctypes.c_int64()
        _lib.check(self.lib.pcm_candidate_stats(self.h, ctypes.byref(mean), ctypes.byref(mx), ctypes.byref(full),
                                                _stream()), "pcm_candidate_stats")
        out = dict(mean=mean.value, max=mx.value, full_cells=full.value)
        z, ft, lt, ll = ctypes.c_int(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        _lib.check(self.lib.pcm_tile_list_stats(self.h, ctypes.byref(z), ctypes.byref(ft), ctypes.byref(lt),
                                                ctypes.byref(ll), _stream()), "pcm_tile_list_stats")
        if z.value > 0:   # crowded layout: tiles of long-list / FULL cells and their own lists
            out.update(zlev=z.value, crowded_tiles=ft.value, listed_tiles=lt.value,
                       tile_list_mean=(ll.value / lt.value) if lt.value else 0.0)
            lg, ak, ml = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
            _lib.check(self.lib.pcm_tile_list_detail(self.h, ctypes.byref(lg), ctypes.byref(ak), ctypes.byref(ml),
                                                     _stream()), "pcm_tile_list_detail")
            out.update(long_tile_lists=lg.value, allk_tiles=ak.value, tile_list_max=ml.value)
        return out


def _dtype_code(X: torch.Tensor) -> int:
    if X.dtype == torch.float32:
        return PCM_F32
    if X.dtype == torch.float16:
        return PCM_F16
    raise ValueError("points dtype must be float32 or float16")


def shard_hist(X: torch.Tensor, axis: int, lo: float, inv: float, nbins: int) -> torch.Tensor:
    """Histogram (int64, device) of bin = clamp(floor((X[:, axis] - lo) * inv)) (``pcm_shard_hist``)."""
    lib = _lib.load()
    X = X.contiguous()
    hist = torch.empty(nbins, dtype=torch.int64, device=X.device)
    _lib.check(lib.pcm_shard_hist(_ptr(X) if X.numel() else None, _dtype_code(X), X.shape[0], X.shape[1], int(axis),
                                  float(lo), float(inv), int(nbins), _ptr(hist), _stream()), "pcm_shard_hist")
    return hist


def shard_partition(X: torch.Tensor, axis: int, lo: float, inv: float, nbins: int, owner, world: int, gidx0: int):
    """Stable partition of the rows by ``owner[bin]`` (``pcm_shard_partition``):
    (rows grouped by destination, their global indices as int32, counts)."""
    lib = _lib.load()
    X = X.contiguous()
    n, d = X.shape
    own = torch.as_tensor(np.ascontiguousarray(owner, dtype=np.uint8), device=X.device)
    out = torch.empty_like(X)
    rows = torch.empty(n, dtype=torch.int32, device=X.device)
    counts = np.zeros(world, dtype=np.int64)
    ws_bytes = ctypes.c_size_t()
    _lib.check(lib.pcm_shard_partition_workspace(n, int(world), ctypes.byref(ws_bytes)), "pcm_shard_partition_workspace")
    ws = torch.empty(max(1, ws_bytes.value), dtype=torch.uint8, device=X.device)
    _lib.check(lib.pcm_shard_partition(_ptr(X) if n else None, _dtype_code(X), n, d, int(axis), float(lo), float(inv),
                                       int(nbins), _ptr(own), int(world), int(gidx0), _ptr(out) if n else None,
                                       _ptr(rows) if n else None, counts.ctypes.data_as(ctypes.c_void_p), _ptr(ws),
                                       ws_bytes.value, _stream()), "pcm_shard_partition")
    return out, rows, counts


def shard_scatter_labels(labels: torch.Tensor, rows: torch.Tensor, gidx0: int, n: int) -> torch.Tensor:
    """out[rows[i] - gidx0] = labels[i] (``pcm_shard_scatter_labels``)."""
    lib = _lib.load()
    out = torch.empty(n, dtype=torch.int32, device=labels.device)
    _lib.check(lib.pcm_shard_scatter_labels(_ptr(labels) if n else None, _ptr(rows) if n else None, int(n), int(gidx0),
                                            _ptr(out) if n else None, _stream()), "pcm_shard_scatter_labels")
    return out


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
