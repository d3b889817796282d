"""Loader and build recipe of the C-ABI HIP library ``libpcmkm.so``.

The library is built in-tree (``build()``), so the shared object travels with
the repository snapshot to the GPU box.  ``load()`` fails loudly when the
library is missing: there is no CPU fallback anywhere in the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
SO_PATH = os.environ.get("PCM_SO") or os.path.join(PKG_DIR, "libpcmkm.so")
UNITS = [os.path.join(PKG_DIR, "csrc", u) for u in ("pcm_engine.hip", "pcm_dense.hip", "pcm_stereo.hip", "pcm_shard.hip",
                                                            "pcm_xchg.hip")]
SOURCES = UNITS + [os.path.join(PKG_DIR, "csrc", h) for h in ("pcm_kernels.hpp", "pcm_kpp.hpp", "pcm_sort.hpp", "pcm_cloud.hpp",
                                                              "pcm_common.hpp", "pcm_debug.hpp", "pcm_xchg.hpp")] + \
    [os.path.join(REPO_DIR, "include", "pcm_kmeans.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
HIP_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared"]

# Every symbol include/pcm_kmeans.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "pcm_abi_version", "pcm_last_error", "pcm_engine_create", "pcm_engine_destroy", "pcm_layout_bbox",
    "pcm_layout_build", "pcm_fit_begin", "pcm_iter_local", "pcm_iter_global", "pcm_iterate", "pcm_stats_ptr",
    "pcm_bind_stats", "pcm_reloc_candidates", "pcm_reloc_apply", "pcm_final", "pcm_labels", "pcm_get_centers",
    "pcm_history", "pcm_read_status", "pcm_status_post", "pcm_status_wait", "pcm_layout_info", "pcm_candidate_stats", "pcm_tile_list_stats", "pcm_tile_list_detail", "pcm_synth_uniform",
    "pcm_assign_bruteforce", "pcm_timing", "pcm_timing_read", "pcm_time_assign", "pcm_synth_rows", "pcm_kmeanspp", "pcm_cloud_assemble",
    "pcm_inertia_value", "pcm_kmeanspp_workspace",
    "pcm_dense_create", "pcm_dense_destroy", "pcm_dense_begin", "pcm_dense_iterate", "pcm_dense_final",
    "pcm_dense_status", "pcm_dense_outputs", "pcm_dense_kmeanspp_workspace", "pcm_dense_kmeanspp",
    "pcm_photoconsistency", "pcm_lr_consistency",
    "pcm_layout_shard", "pcm_shard_hist", "pcm_shard_partition_workspace", "pcm_shard_partition",
    "pcm_shard_scatter_labels", "pcm_assign_kernel_name", "pcm_layout_stream_bytes", "pcm_engine_reserve",
    "pcm_xchg_create", "pcm_xchg_destroy", "pcm_xchg_handle", "pcm_xchg_open", "pcm_xchg_link", "pcm_xchg_allreduce",
    "pcm_xchg_status", "pcm_iter_exchange",
]
ABI_VERSION = 6

_lock = threading.Lock()
_lib = None


class PcmError(RuntimeError):
    pass


class PcmStatus(ctypes.Structure):
    _fields_ = [("halt", ctypes.c_uint32), ("done", ctypes.c_uint32), ("iter", ctypes.c_uint32),
                ("n_empty", ctypes.c_uint32), ("inertia", ctypes.c_double), ("last_changed", ctypes.c_uint64),
                ("last_shift", ctypes.c_double), ("inertia_limbs", ctypes.c_uint64 * 3),
                ("inertia_scale", ctypes.c_int32), ("inertia_overflow", ctypes.c_uint32),
                ("list_rebuilds", ctypes.c_uint32), ("pad_", ctypes.c_uint32)]


def needs_build() -> bool:
    if not os.path.exists(SO_PATH):
        return True
    t = os.path.getmtime(SO_PATH)
    return any(os.path.getmtime(s) > t for s in SOURCES if os.path.exists(s))


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile ``libpcmkm.so`` for gfx950 with hipcc (works without a GPU)."""
    if not force and not needs_build():
        return SO_PATH
    # the translation units compile in parallel (-c) into an object cache outside
    # the tree (a unit is rebuilt when it or a header it includes is newer than
    # its object), then one link
    import re
    from concurrent.futures import ThreadPoolExecutor
    inc = ["-I", os.path.join(REPO_DIR, "include")]
    objdir = os.environ.get("PCM_OBJ_DIR") or os.path.join("/tmp", "pcm_build_objs")
    os.makedirs(objdir, exist_ok=True)

    def deps(path, seen):
        if path in seen or not os.path.exists(path):
            return seen
        seen.add(path)
        for h in re.findall(r'#include\s+"([^"]+)"', open(path).read()):
            for d in (os.path.dirname(path), os.path.join(REPO_DIR, "include")):
                if os.path.exists(os.path.join(d, h)):
                    deps(os.path.join(d, h), seen)
                    break
        return seen

    objs, cmds = [], []
    for u in UNITS:
        o = os.path.join(objdir, os.path.basename(u) + ".o")
        objs.append(o)
        if force or not os.path.exists(o) or any(os.path.getmtime(d) > os.path.getmtime(o) for d in deps(u, set())):
            cmds.append([HIPCC, *HIP_FLAGS[:-1], *inc, "-c", u, "-o", o])
    if verbose:
        print("\n".join(" ".join(c) for c in cmds))
    with ThreadPoolExecutor(max_workers=max(1, min(len(cmds), os.cpu_count() or 1))) as ex:
        for r in list(ex.map(lambda c: subprocess.run(c, capture_output=not verbose, text=True), cmds)):
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed:\n{' '.join(r.args)}\n{r.stdout or ''}{r.stderr or ''}")
    link = [HIPCC, "--offload-arch=gfx950", "-fPIC", "-shared", "-o", SO_PATH + ".tmp", *objs]
    subprocess.run(link, check=True)
    os.replace(SO_PATH + ".tmp", SO_PATH)
    return SO_PATH


def _declare(lib):
    P, I, I64, D = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_double
    sig = {
        "pcm_abi_version": ([], I),
        "pcm_last_error": ([ctypes.c_char_p, ctypes.c_size_t], I),
        "pcm_engine_create": ([I, I, I, I, I, ctypes.POINTER(P)], I),
        "pcm_engine_destroy": ([P], I),
        "pcm_layout_bbox": ([P, P, I64, P, P, P, P], I),
        "pcm_layout_build": ([P, P, P, I64, P], I),
        "pcm_engine_reserve": ([P, I64, P], I),
        "pcm_fit_begin": ([P, P, D, I, P], I),
        "pcm_iter_local": ([P, P], I),
        "pcm_iter_global": ([P, P], I),
        "pcm_iterate": ([P, I, P], I),
        "pcm_stats_ptr": ([P, ctypes.POINTER(P), ctypes.POINTER(I64)], I),
        "pcm_bind_stats": ([P, P], I),
        "pcm_reloc_candidates": ([P, I, P, P], I),
        "pcm_reloc_apply": ([P, P, I, P], I),
        "pcm_final": ([P, P], I),
        "pcm_labels": ([P, P, P], I),
        "pcm_time_assign": ([P, I, P, ctypes.POINTER(D)], I),
        "pcm_get_centers": ([P, P, P], I),
        "pcm_history": ([P, P, P, I, P], I),
        "pcm_read_status": ([P, ctypes.POINTER(PcmStatus), P], I),
        "pcm_status_post": ([P, P], I),
        "pcm_status_wait": ([P, ctypes.POINTER(PcmStatus)], I),
        "pcm_layout_info": ([P, ctypes.POINTER(I64), ctypes.POINTER(I64), P], I),
        "pcm_candidate_stats": ([P, ctypes.POINTER(D), ctypes.POINTER(I), ctypes.POINTER(I64), P], I),
        "pcm_tile_list_stats": ([P, ctypes.POINTER(I), ctypes.POINTER(I64), ctypes.POINTER(I64), ctypes.POINTER(I64), P],
                                I),
        "pcm_tile_list_detail": ([P, ctypes.POINTER(I64), ctypes.POINTER(I64), ctypes.POINTER(I64), P], I),
        "pcm_synth_uniform": ([P, I64, I, ctypes.c_uint64, I64, P], I),
        "pcm_assign_bruteforce": ([P, I64, I, P, I, P, P, P, P], I),
        "pcm_timing": ([P, I], I),
        "pcm_timing_read": ([P, P, ctypes.POINTER(I)], I),
        "pcm_synth_rows": ([P, P, I64, I, ctypes.c_uint64, P], I),
        "pcm_kmeanspp": ([P, I64, I, I, I, I64, P, P, P, ctypes.c_size_t, P], I),
        "pcm_kmeanspp_workspace": ([I64, I, I, I, ctypes.POINTER(ctypes.c_size_t)], I),
        "pcm_cloud_assemble": ([P, P, I64, I64, D, P, P, ctypes.POINTER(I64), P, P], I),
        "pcm_inertia_value": ([P, I, ctypes.c_uint32], D),
        "pcm_dense_create": ([I, I64, I, I, I, I, ctypes.POINTER(P)], I),
        "pcm_dense_destroy": ([P], I),
        "pcm_dense_begin": ([P, P, P, P, D, I, P], I),
        "pcm_dense_iterate": ([P, I, P], I),
        "pcm_dense_final": ([P, P], I),
        "pcm_dense_status": ([P, ctypes.POINTER(PcmStatus), P], I),
        "pcm_dense_outputs": ([P, P, P, P, P, I, P], I),
        "pcm_dense_kmeanspp_workspace": ([I64, I, I, I, I, ctypes.POINTER(ctypes.c_size_t)], I),
        "pcm_dense_kmeanspp": ([P, I64, I, I, I, I, I64, P, I, P, P, ctypes.c_size_t, P], I),
        "pcm_photoconsistency": ([P, P, I, P, I64, I64, D, P, P], I),
        "pcm_lr_consistency": ([P, P, I64, I64, D, D, P, P, D, P], I),
        "pcm_layout_shard": ([P, P, I64, P], I),
        "pcm_shard_hist": ([P, I, I64, I, I, D, D, I, P, P], I),
        "pcm_shard_partition_workspace": ([I64, I, ctypes.POINTER(ctypes.c_size_t)], I),
        "pcm_shard_partition": ([P, I, I64, I, I, D, D, I, P, I, I64, P, P, P, P, ctypes.c_size_t, P], I),
        "pcm_shard_scatter_labels": ([P, P, I64, I64, P, P], I),
        "pcm_assign_kernel_name": ([P, ctypes.c_char_p, ctypes.c_size_t], I),
        "pcm_layout_stream_bytes": ([P, ctypes.POINTER(D), ctypes.POINTER(I64)], I),
        "pcm_xchg_create": ([I, I64, I, I, D, ctypes.POINTER(P)], I),
        "pcm_xchg_destroy": ([P], I),
        "pcm_xchg_handle": ([P, P], I),
        "pcm_xchg_open": ([P, I, P], I),
        "pcm_xchg_link": ([P, I, P], I),
        "pcm_xchg_allreduce": ([P, P, I, P], I),
        "pcm_xchg_status": ([P, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64), P], I),
        "pcm_iter_exchange": ([P, P, I, P], I),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res


def load(require_gpu_runtime: bool = True):
    """Load the library (after torch, so one HIP runtime serves both)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(SO_PATH):
                raise PcmError(f"HIP extension missing: {SO_PATH} (run __graft_entry__.build())")
            if require_gpu_runtime:
                import torch  # noqa: F401  (loads torch's libamdhip64.so.7 first)
            lib = ctypes.CDLL(SO_PATH)
            _declare(lib)
            _lib = lib
    return _lib


def last_error() -> str:
    buf = ctypes.create_string_buffer(1024)
    load().pcm_last_error(buf, 1024)
    return buf.value.decode(errors="replace")


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        raise PcmError(f"{what} failed ({rc}): {last_error()}")
