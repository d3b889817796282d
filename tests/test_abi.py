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


def test_exchange_argument_errors_without_device(lib):
    """The peer exchange's argument checks run before any device call."""
    from pcm_amd import _lib
    h = ctypes.c_void_p()
    assert lib.pcm_xchg_create(0, 0, 2, 0, 1.0, ctypes.byref(h)) == -1        # no words
    assert lib.pcm_xchg_create(0, 8, 17, 0, 1.0, ctypes.byref(h)) == -1       # > PCM_XCHG_MAXP ranks
    assert lib.pcm_xchg_create(0, 8, 2, 2, 1.0, ctypes.byref(h)) == -1        # rank out of range
    assert lib.pcm_xchg_create(0, 8, 2, 0, 0.0, ctypes.byref(h)) == -1        # no timeout
    assert "pcm_xchg_create" in _lib.last_error()
    assert lib.pcm_iter_exchange(None, None, 3, None) == -1
    assert lib.pcm_xchg_allreduce(None, None, 3, None) == -1
    assert lib.pcm_xchg_destroy(None) == 0


def test_exchange_choice_host_logic():
    """xchg.choose / lloyd.exchange_for without a device: one rank or the
    collective mode never builds an exchange; unknown modes are rejected."""
    from pcm_amd import lloyd, xchg
    assert xchg.choose("collective", 8, 4, None, None) is None
    assert xchg.choose("peer", 8, 1, None, None) is None
    with pytest.raises(ValueError):
        xchg.choose("rdma", 8, 4, None, None)

    class Stub:
        stats = None
    assert lloyd.exchange_for(Stub(), "auto") is None          # world 1 (no process group)


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
