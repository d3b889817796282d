"""CPU: the C-ABI library loads and exports every symbol include/pcm_kmeans.h declares.

No compute calls (there is no GPU here); argument validation paths that fail
before touching the device are exercised.
"""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pcm_kmeans.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(?:int|double)\s+(pcm_\w+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from pcm_amd import _lib
    if not os.path.exists(_lib.SO_PATH):
        _lib.build()
    return _lib.load(require_gpu_runtime=False)


def test_header_declares_expected_entry_points():
    from pcm_amd import _lib
    assert declared() == sorted(_lib.EXPORTS)


def test_every_declared_symbol_is_exported(lib):
    for name in declared():
        assert hasattr(lib, name), name


def test_abi_version(lib):
    from pcm_amd import _lib
    assert lib.pcm_abi_version() == _lib.ABI_VERSION


def test_argument_errors_without_device(lib):
    from pcm_amd import _lib
    h = ctypes.c_void_p()
    assert lib.pcm_engine_create(0, 7, 8, 0, 10, ctypes.byref(h)) == -1     # d out of range
    assert "d must be" in _lib.last_error()
    assert lib.pcm_engine_create(0, 3, 0, 0, 10, ctypes.byref(h)) == -1     # k < 1
    assert lib.pcm_engine_create(0, 3, 8, 5, 10, ctypes.byref(h)) == -1     # bad dtype
    assert lib.pcm_synth_uniform(None, -1, 3, 0, 0, None) == -1
    assert lib.pcm_iter_local(None, None) == -1


def test_no_fp_contraction_in_build_flags():
    from pcm_amd import _lib
    assert "-ffp-contract=off" in _lib.HIP_FLAGS
    assert "--offload-arch=gfx950" in _lib.HIP_FLAGS


def test_inertia_value_from_limbs(lib):
    """pcm_inertia_value: exact integer total, one rounding, exact scaling (host only)."""
    import math
    limbs = (ctypes.c_uint64 * 3)(0xFFFFFFFF, 0xFFFFFFFF, 12345)
    total = 0xFFFFFFFF + (0xFFFFFFFF << 32) + (12345 << 64)
    assert lib.pcm_inertia_value(limbs, 70, 0) == math.ldexp(float(total), -70)
    assert lib.pcm_inertia_value(limbs, 0, 1) == float("inf")
