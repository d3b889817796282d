"""One-sided cross-rank SUM of the Lloyd statistics (``csrc/pcm_xchg.hip``).

The multi-GPU iteration (``lloyd.run``) sums every rank's K*(D+1)+1 integer
statistics between the assign kernel and the update.  ``PeerExchange`` does it
without a collective: each rank pushes its statistics into a slot of every
peer's receive buffer (IPC-mapped device memory), raises a flag there, and sums
the slots its peers pushed once their flags arrive -- two small kernels on the
rank's own stream, no host involvement, capturable in a HIP graph with any
process-group backend.  Integer sums make the result bit-identical to the RCCL
all-reduce it replaces.

Setup is collective: every rank creates its exchange, the IPC handles are
all-gathered over the process group, every rank maps its peers' buffers and a
self-test (two exchanges of a known pattern, one per buffer parity) must give
the exact sum on every rank.  Any failure on any rank makes every rank fall
back to the collective (``exchange="auto"``) or raise (``"peer"``).
"""
from __future__ import annotations

import ctypes
import os
import warnings

import torch

from . import _lib

HANDLE_BYTES = 64
MAXP = 16


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class PeerExchange:
    """This rank's end of the exchange: ``words`` int64 summed over ``world`` ranks."""

    def __init__(self, words: int, world: int, rank: int, device=None, timeout_s: float = None):
        self.lib = _lib.load()
        self.words, self.world, self.rank = int(words), int(world), int(rank)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else torch.device(device).index)
        if timeout_s is None:
            timeout_s = float(os.environ.get("PCM_XCHG_TIMEOUT_S", "20"))
        h = ctypes.c_void_p()
        _lib.check(self.lib.pcm_xchg_create(self.device.index, self.words, self.world, self.rank, float(timeout_s),
                                            ctypes.byref(h)), "pcm_xchg_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.pcm_xchg_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def handle(self) -> bytes:
        buf = ctypes.create_string_buffer(HANDLE_BYTES)
        _lib.check(self.lib.pcm_xchg_handle(self.h, buf), "pcm_xchg_handle")
        return buf.raw

    def open(self, peer: int, handle: bytes):
        buf = ctypes.create_string_buffer(bytes(handle), HANDLE_BYTES)
        _lib.check(self.lib.pcm_xchg_open(self.h, int(peer), buf), "pcm_xchg_open")

    def link(self, peer: int, other: "PeerExchange"):
        _lib.check(self.lib.pcm_xchg_link(self.h, int(peer), other.h), "pcm_xchg_link")

    def allreduce(self, buf: torch.Tensor, phase: int = 3):
        """buf (device int64[words]) := SUM over the ranks, in place (stream-ordered)."""
        if buf.dtype != torch.int64 or buf.numel() != self.words or not buf.is_contiguous():
            raise ValueError("buf must be a contiguous int64 tensor of `words` elements")
        _lib.check(self.lib.pcm_xchg_allreduce(self.h, ctypes.c_void_p(buf.data_ptr()), int(phase), _stream()),
                   "pcm_xchg_allreduce")

    def status(self) -> dict:
        err, ep = ctypes.c_uint32(), ctypes.c_uint64()
        _lib.check(self.lib.pcm_xchg_status(self.h, ctypes.byref(err), ctypes.byref(ep), _stream()), "pcm_xchg_status")
        return dict(err=int(err.value), epoch=int(ep.value))


def _pattern(rank: int, words: int, salt: int, device) -> torch.Tensor:
    i = torch.arange(words, dtype=torch.int64, device=device)
    return (i * 7919 + (rank + 1) * 1_000_003 + salt * (1 << 40)) ^ (rank << 17)


def self_test(x: PeerExchange, device) -> bool:
    """Two exchanges of a known pattern (both buffer parities): the exact sum on this rank?"""
    ok = True
    for salt in (1, 2):
        buf = _pattern(x.rank, x.words, salt, device)
        want = sum(_pattern(r, x.words, salt, device) for r in range(x.world))
        x.allreduce(buf)
        torch.cuda.synchronize()
        ok = ok and bool(torch.equal(buf, want))
    return ok and x.status()["err"] == 0


def setup(words: int, group=None, device=None, timeout_s: float = None):
    """Collective: a verified PeerExchange on every rank, or None on every rank
    (a failure anywhere -- creation, IPC mapping, self-test -- is agreed over
    ``group``).  Returns (exchange or None, reason)."""
    import torch.distributed as dist

    from .lloyd import agree
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    if world > MAXP:
        return None, f"world size {world} > {MAXP}"
    x, err = None, None
    try:
        x = PeerExchange(words, world, rank, dev, timeout_s)
        mine = torch.frombuffer(bytearray(x.handle()), dtype=torch.uint8).to(dev)
    except Exception as exc:   # noqa: BLE001 -- agreed below
        err, mine = exc, torch.zeros(HANDLE_BYTES, dtype=torch.uint8, device=dev)
    if not agree(err is None, world, group, dev):
        return None, f"create: {err!r}" if err is not None else "create failed on another rank"
    parts = [torch.zeros(HANDLE_BYTES, dtype=torch.uint8, device=dev) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    try:
        for r in range(world):
            if r != rank:
                x.open(r, parts[r].cpu().numpy().tobytes())
    except Exception as exc:   # noqa: BLE001
        err = exc
    if not agree(err is None, world, group, dev):
        return None, f"open: {err!r}" if err is not None else "IPC open failed on another rank"
    try:
        ok = self_test(x, dev)
    except Exception as exc:   # noqa: BLE001
        ok, err = False, exc
    if not agree(ok, world, group, dev):
        return None, f"self-test: {err!r}" if err is not None else "self-test failed"
    return x, "ok"


def linked(words: int, world: int, device=None, timeout_s: float = None):
    """``world`` exchanges of ONE process linked to each other (the 1-GPU slab
    proxy of bench.py: every "rank" is an engine of this process)."""
    xs = [PeerExchange(words, world, r, device, timeout_s) for r in range(world)]
    for r, x in enumerate(xs):
        for p, y in enumerate(xs):
            if p != r:
                x.link(p, y)
    return xs


def choose(mode: str, words: int, world: int, group, device):
    """The exchange ``lloyd.run`` uses: ``mode`` "collective" -> None; "peer" ->
    a verified PeerExchange or raise; "auto" -> PeerExchange when it verifies on
    every rank, else None with a warning.  PCM_XCHG=0 forces the collective."""
    if mode not in ("auto", "peer", "collective"):
        raise ValueError("exchange must be 'auto', 'peer' or 'collective'")
    if world <= 1 or mode == "collective" or (mode == "auto" and os.environ.get("PCM_XCHG", "1") == "0"):
        return None
    x, why = setup(words, group, device)
    if x is None:
        if mode == "peer":
            raise _lib.PcmError(f"peer exchange unavailable: {why}")
        warnings.warn(f"pcm_amd: peer exchange unavailable ({why}); using the process-group all-reduce")
    return x


__all__ = ["PeerExchange", "setup", "linked", "choose", "self_test"]
