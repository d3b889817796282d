"""ctypes binding of oracle/lloyd_ref.c (TEST INFRASTRUCTURE ONLY, see lloyd_ref.py)."""
from __future__ import annotations


import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liblloydref.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        lib = ctypes.CDLL(_SO)
        P = ctypes.c_void_p
        lib.ref_lloyd_stats.argtypes = [P, ctypes.c_int64, ctypes.c_int, P, ctypes.c_int,
                                        P, P, P, P, P, ctypes.c_int]
        lib.ref_lloyd_stats.restype = ctypes.c_int64
        lib.ref_max_threads.restype = ctypes.c_int
        _lib = lib
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def lloyd_stats(X, C, q=None, labels_old=None, nthreads=None, with_sums=True):
    """Returns (labels, sums (k,d) int64, counts (k,) int64, n_changed)."""
    lib = load()
    X = np.ascontiguousarray(X, dtype=np.float32)
    C = np.ascontiguousarray(C, dtype=np.float32)
    n, d = X.shape
    k = C.shape[0]
    if q is None:
        q = np.zeros(d, dtype=np.int32)
    q = np.ascontiguousarray(q, dtype=np.int32)
    lo = None if labels_old is None else np.ascontiguousarray(labels_old, dtype=np.int32)
    labels = np.empty(n, dtype=np.int32)
    sums = np.zeros((k, d), dtype=np.int64) if with_sums else None
    counts = np.zeros(k, dtype=np.int64) if with_sums else None
    nt = nthreads or lib.ref_max_threads()
    nch = lib.ref_lloyd_stats(_p(X), n, d, _p(C), k, _p(q), _p(lo), _p(labels),
                              _p(sums), _p(counts), int(nt))
    return labels, sums, counts, int(nch)
