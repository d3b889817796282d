"""Lloyd K-means fit driver: one process per GPU, row-sharded cloud.

Restates the control flow of scikit-learn's ``_kmeans_single_lloyd``
(sklearn/cluster/_kmeans.py:623-752) over the C-ABI engine:

* the loop body (E-step + M-step, ``lloyd_iter_chunked_dense``,
  _k_means_lloyd.pyx:23-165) is ``Engine.iter_local`` (candidate lists, assign,
  exact integer accumulation) + an all-reduce of the integer statistics +
  ``Engine.iter_global`` (relocation check, averaging, shift, convergence);
* strict label convergence / shift tolerance (``_kmeans.py:717-732``) are
  evaluated on the device; iterations are enqueued in chunks with one host
  synchronisation per chunk (iterations queued past convergence are no-ops);
* empty clusters (``_k_means_common.pyx:167-211``) halt the device loop; the
  host gathers every rank's farthest points and resumes;
* the final E-step + inertia (``_kmeans.py:736-750``) is ``Engine.final``.

Multi-GPU: rank r receives a contiguous row shard; at layout time the shards are
regrouped into equal-count spatial slabs (one all_to_all of the points; the
labels travel back after the final E-step).  Per iteration the ranks sum
K*(D+1)+1 int64 statistics: by the one-sided peer exchange (``xchg.py``: writes
into the peers' memory over xGMI, no collective) or by one SUM all-reduce
(RCCL with the ``nccl`` backend).  Integer statistics make the result
bit-identical for any world size, sharding and exchange.
"""
from __future__ import annotations

import warnings
from dataclasses import dataclass, field

import numpy as np
import torch

from .fixed import fixed_q, inertia_from_limbs


@dataclass
class LloydResult:
    labels: torch.Tensor          # this rank's rows, original order, int32
    centers: torch.Tensor         # (K, D) float32
    inertia: float                # global
    n_iter: int
    strict: bool                  # converged by label equality
    # per iteration: how many of the K*(D+1) integer statistic words differ from the
    # previous iteration's -- NOT sklearn's count of changed labels (the engine never
    # stores per-point labels while iterating); 0 exactly when no label
    # changed, which is when sklearn's strict convergence fires (_kmeans.py:717-722)
    stat_words_changed: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int64))
    shift: np.ndarray = field(default_factory=lambda: np.zeros(0))
    relocations: int = 0
    layout: dict = field(default_factory=dict)


class _Local:
    """``group=LOCAL``: a single-process fit even when a default process group
    exists (the estimator and the plugin fit the whole cloud on one GPU)."""

    def __repr__(self):
        return "pcm_amd.lloyd.LOCAL"


LOCAL = _Local()


def _world(group):
    import torch.distributed as dist
    if group is LOCAL:
        return 1, 0
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


XCHG_FAILED = 4     # pcm_status.done: a peer exchange timed out
UPD_FAILED = 5      # pcm_status.done: k_updlists' publisher timed out waiting for its list blocks
SLAB_BINS = 16384   # slab histogram resolution (pcm_shard_hist's LDS bound)
SLAB_MAXP = 16      # PCM_SHARD_MAXP: ranks a slab partition can address (uint8 owner table, LDS counters)


def slab_sizes(hist: np.ndarray, owner: np.ndarray, world: int) -> np.ndarray:
    """Points each rank's slab receives (from the all-reduced histogram and the
    owner table every rank holds: the same numbers on every rank)."""
    return np.bincount(np.asarray(owner, np.int64), weights=np.asarray(hist, np.float64),
                       minlength=world).astype(np.int64)


def _agreed(fn, what, world, group, device):
    """fn() on every rank; a failure on any rank raises on every rank (MIN
    all-reduce of an ok flag), so no rank is left waiting in the next collective."""
    err, out = None, None
    try:
        out = fn()
    except Exception as exc:   # noqa: BLE001 -- re-raised below, after the ranks agree
        err = exc
    if not agree(err is None, world, group, device):
        if err is not None:
            raise err
        raise RuntimeError(f"pcm_amd.lloyd: {what} failed on another rank")
    return out


def _build_all(engine, X, q, gidx0, world, group):
    """engine.build on every rank, failures agreed (``_agreed``)."""
    _agreed(lambda: engine.build(X, q, gidx0), "the layout build", world, group, engine.stats_device)


def slab_owner(hist: np.ndarray, world: int) -> np.ndarray:
    """Bin -> rank of the equal-count slab cut: bin b goes to the rank whose
    share [r N / P, (r + 1) N / P) holds the bin's midpoint count.  Monotone in
    b, so every rank owns one contiguous slab of the axis."""
    h = np.asarray(hist, dtype=np.int64)
    total = int(h.sum())
    if total == 0:
        return np.zeros(h.shape[0], np.uint8)
    before = np.cumsum(h) - h
    return np.minimum(world - 1, ((2 * before + h) * world) // (2 * total)).astype(np.uint8)


def prepare(engine, X, group=None, shard: str = "auto"):
    """Layout phase: global fixed-point exponents, shard offsets, cell sort.

    ``shard`` (world > 1): "slab" (= "auto") regroups the ranks' row shards into
    equal-count slabs of the longest axis of the global bounding box (one
    all_to_all of the points at layout time; labels travel back in ``finish``),
    so each rank's pruning grid covers only its slab and its per-iteration work
    shrinks with the world size; "rows" keeps the row shards in place."""
    import torch.distributed as dist
    world, rank = _world(group)
    n_local = int(X.shape[0])
    lo, hi, maxabs = engine.bbox(X)
    engine._slab = None
    if world == 1:
        q = fixed_q(maxabs)
        engine.build(X, q, 0)
        return q, n_local
    if shard not in ("auto", "slab", "rows"):
        raise ValueError("shard must be 'auto', 'slab' or 'rows'")
    if world > SLAB_MAXP:
        if shard == "slab":
            raise ValueError(f"shard='slab' supports at most {SLAB_MAXP} ranks (world size {world}); use 'rows'")
        shard = "rows"      # 'auto': row shards work at any world size
    dev = engine.stats_device
    mine = torch.tensor([n_local], dtype=torch.int64, device=dev)
    parts = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    counts = [int(p.item()) for p in parts]
    gidx0, n_total = sum(counts[:rank]), sum(counts)
    if n_total >= 2 ** 32:
        raise ValueError("at most 2**32 - 1 points in one fit")
    lo = np.asarray(lo, np.float64) if n_local else np.full(engine.d, np.inf)
    hi = np.asarray(hi, np.float64) if n_local else np.full(engine.d, -np.inf)
    m = torch.tensor(np.concatenate([-lo, hi, np.asarray(maxabs, np.float64)]), device=dev)
    dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
    m = m.cpu().numpy()
    d = engine.d
    glo, ghi, maxabs = -m[:d], m[d:2 * d], m[2 * d:]
    q = fixed_q(maxabs)
    if shard == "rows" or n_total == 0:
        _build_all(engine, X, q, gidx0, world, group)
        return q, n_total
    ext = ghi - glo
    axis = int(np.argmax(ext))
    inv = SLAB_BINS / ext[axis] if ext[axis] > 0 else 0.0
    hist = engine.shard_hist(X, axis, glo[axis], inv, SLAB_BINS)
    dist.all_reduce(hist, group=group)
    hist_h = hist.cpu().numpy()
    owner = slab_owner(hist_h, world)
    from .engine import ENGINE_MAX_POINTS
    if int(slab_sizes(hist_h, owner, world).max()) > ENGINE_MAX_POINTS:
        # a dense bin would overfill one rank's engine: every rank sees the same
        # histogram and owner table, so all of them keep their row shards together
        warnings.warn("pcm_amd.lloyd: a spatial slab would exceed one engine's capacity; keeping row shards")
        _build_all(engine, X, q, gidx0, world, group)
        return q, n_total
    # every step that can fail on one rank alone (a partition workspace or a receive
    # buffer out of memory on a skewed rank) is agreed before the next collective
    sdev = engine.stats_device
    Xs, rows, send = _agreed(lambda: engine.shard_partition(X, axis, glo[axis], inv, SLAB_BINS, owner, world, gidx0),
                             "the slab partition", world, group, sdev)
    st = torch.tensor(send, dtype=torch.int64, device=dev)
    rt = torch.empty_like(st)
    dist.all_to_all_single(rt, st, group=group)
    recv = rt.cpu().numpy().astype(np.int64)
    sl, rl = [int(v) for v in send], [int(v) for v in recv]
    Xr, rows_r = _agreed(lambda: (torch.empty((sum(rl), d), dtype=X.dtype, device=X.device),
                                  torch.empty(sum(rl), dtype=torch.int32, device=X.device)),
                         "the slab receive buffers", world, group, sdev)
    dist.all_to_all_single(Xr, Xs, rl, sl, group=group)
    dist.all_to_all_single(rows_r, rows, rl, sl, group=group)
    del Xs
    _agreed(lambda: (engine.bbox(Xr), engine.set_shard(rows_r, n_total)), "the slab bounding box", world, group,
            sdev)
    _build_all(engine, Xr, q, 0, world, group)
    engine._slab = dict(rows=rows, send=sl, recv=rl, gidx0=gidx0, n_local=n_local, axis=axis,
                        n_slab=sum(rl))
    return q, n_total


def _uses_graph(graph, world, group, split, xchg=None):
    """HIP-graph replay of the multi-GPU iteration sequence.  With the peer
    exchange (``xchg``) the sequence holds no collective: captured by default,
    on any backend (``graph=False`` or ``PCM_LLOYD_GRAPH=0`` launches eagerly).
    With the collective all-reduce only RCCL's collectives can be captured
    (gloo's cannot), and since round 6 that capture is opt-in (``graph=True`` or
    ``PCM_LLOYD_GRAPH=1``): the collective is now the fallback path, and a
    captured multi-rank RCCL sequence has no multi-GPU run on record.
    A refused capture falls back to eager launches on every rank (``agree``)."""
    import os

    import torch.distributed as dist
    env = os.environ.get("PCM_LLOYD_GRAPH")
    if not (world > 1 or split) or not dist.is_initialized():
        return False
    if xchg is not None:
        return graph is not False and env != "0"
    if not (graph is True or (graph is None and env == "1")):
        return False
    try:
        return dist.get_backend(group) == "nccl"
    except Exception:   # noqa: BLE001
        return False


def agree(ok: bool, world: int, group=None, device=None) -> bool:
    """True only if ``ok`` holds on every rank (MIN all-reduce of a flag), so that
    all ranks take the same path (captured graph vs eager launches) and their
    collective sequences stay aligned."""
    if world <= 1:
        return ok
    import torch.distributed as dist
    t = torch.tensor([1 if ok else 0], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


def run(engine, C0, max_iter=300, tol=0.0, group=None, chunk=8, split=False, graph=None, xchg=None):
    """Iteration phase on a prepared engine.  Returns (status, relocations).

    ``xchg``: a verified ``xchg.PeerExchange`` of this rank (world > 1), which
    sums the statistics over the ranks by peer-memory writes in place of
    ``dist.all_reduce`` (the sequence then holds no collective).

    One process: ``pcm_iterate`` (k_lloyd + fused k_step per iteration).  Several
    (or ``split``): ``iter_local`` (k_lloyd accumulating into the statistics
    buffer) -> all-reduce of the statistics (only when world > 1) ->
    ``iter_global`` (k_step on them).  With RCCL (and ``graph`` not False, see
    ``_uses_graph``) a chunk of that sequence is captured once in a HIP graph and replayed: no host launch
    gaps between the kernels and the collective; the device control block gates
    iterations queued past convergence or a halt either way."""
    import torch
    import torch.distributed as dist
    world, _ = _world(group)
    engine.begin(C0, tol, max_iter)
    relocs = 0
    it = 0
    use_graph = _uses_graph(graph, world, group, split, xchg)
    captured = None

    def seq(n):
        for _ in range(n):
            engine.iter_local()
            if xchg is not None:
                engine.exchange(xchg)
            elif world > 1:
                dist.all_reduce(engine.stats, group=group)
            engine.iter_global()

    def check(st):
        if st["done"] == XCHG_FAILED:
            from ._lib import PcmError
            raise PcmError("pcm_amd.lloyd: the peer statistics exchange timed out (a rank stopped pushing); "
                           "the fit is void")
        if st["done"] == UPD_FAILED:
            from ._lib import PcmError
            raise PcmError("pcm_amd.lloyd: the update's publisher timed out waiting for its list blocks; "
                           "the fit is void")

    import os
    if world == 1 and not split and hasattr(engine, "status_post") and os.environ.get("PCM_LLOYD_PIPE", "1") != "0":
        # One GPU: the next chunk is queued before the previous chunk's status is
        # read (a pinned snapshot + event behind each chunk), so the GPU does not
        # idle through the host round trip.  Iterations queued past convergence,
        # max_iter or a halt are gated no-ops on the device (ctrl), and a gated
        # iteration does not advance ctrl.iter, so nothing is lost or repeated.
        queued = min(chunk, max_iter)
        engine.iterate(queued)
        engine.status_post()
        while True:
            spec = min(chunk, max_iter - queued)
            if spec > 0:
                engine.iterate(spec)   # queued behind the snapshot
                queued += spec
            st = engine.status_wait()  # the status before that chunk
            check(st)
            if st["halt"]:
                # the queued chunk ran gated; the relocation follows it in stream order
                recs = engine.reloc_candidates(int(st["n_empty"]))
                engine.reloc_apply(recs)
                relocs += 1
                st = engine.status()
                check(st)
                if st["done"]:
                    return st, relocs
                queued = int(st["iter"])   # nothing in flight: count from the device
                n = min(chunk, max_iter - queued)
                engine.iterate(n)
                queued += n
                engine.status_post()
                continue
            if st["done"]:
                return st, relocs
            if spec == 0:   # every iteration was queued before the snapshot (max_iter gates the rest)
                st = engine.status()
                check(st)
                return st, relocs
            engine.status_post()   # the status after the chunk just queued

    while True:
        n_enq = max(1, min(chunk, max_iter - it))
        if world == 1 and not split:
            engine.iterate(n_enq)
        elif use_graph and n_enq == chunk:
            if captured is None:
                ok = True
                try:
                    captured = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(captured):
                        seq(chunk)
                except Exception as exc:   # noqa: BLE001 -- capture refused: eager launches
                    ok = False
                    warnings.warn(f"pcm_amd.lloyd: HIP-graph capture failed ({exc!r}); eager launches")
                    torch.cuda.synchronize()
                # every rank takes the same path (capture records the collectives without running them)
                if not agree(ok, world, group, engine.stats_device):
                    captured, use_graph = None, False
                    seq(n_enq)
            if captured is not None:
                captured.replay()
        else:
            seq(n_enq)
        st = engine.status()
        check(st)
        if st["halt"]:
            recs = engine.reloc_candidates(int(st["n_empty"]))
            if world > 1:
                parts = [torch.empty_like(recs) for _ in range(world)]
                dist.all_gather(parts, recs, group=group)
                recs = torch.cat(parts)
            engine.reloc_apply(recs)
            relocs += 1
            st = engine.status()
        it = int(st["iter"])
        if st["done"]:
            return st, relocs


def finish(engine, group=None):
    import torch.distributed as dist
    world, _ = _world(group)
    engine.final()
    labels = engine.labels()
    sl = getattr(engine, "_slab", None)
    if sl is not None:
        # the slab's labels travel back to the ranks that own the rows (reverse all_to_all),
        # then into the caller's row order
        back = torch.empty(sl["n_local"], dtype=torch.int32, device=labels.device)
        dist.all_to_all_single(back, labels, sl["send"], sl["recv"], group=group)
        labels = engine.shard_scatter_labels(back, sl["rows"], sl["gidx0"], sl["n_local"])
    st = engine.status()
    inertia = st["inertia"]
    if world > 1:   # exact integer limbs: the same inertia for any world size
        t = torch.tensor(list(st["inertia_limbs"]) + [st["inertia_overflow"]], dtype=torch.int64,
                         device=engine.stats_device)
        dist.all_reduce(t, group=group)
        v = [int(x) for x in t.cpu().tolist()]
        inertia = inertia_from_limbs(v[:3], st["inertia_scale"], v[3])
    return labels, engine.centers(), inertia


def exchange_for(engine, mode: str, group=None):
    """The statistics exchange of a multi-rank fit (``xchg.choose``), kept on the
    engine so that later fits reuse it (its setup maps the peers' buffers and
    runs a self-test).  None: the process-group all-reduce."""
    world, rank = _world(group)
    if world <= 1 or mode == "collective" or not getattr(engine, "h", None):
        return None
    key = (mode, world, rank, id(group))
    cached = getattr(engine, "_xchg", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    from . import xchg
    cnt = engine.stats.numel()
    x = xchg.choose(mode, cnt, world, group, engine.stats_device)
    engine._xchg = (key, x)
    return x


def lloyd_fit(X, centers_init, max_iter: int = 300, tol: float = 0.0, *, group=None, chunk: int = 8,
              engine=None, split: bool = False, graph=None, shard: str = "auto",
              exchange: str = "auto") -> LloydResult:
    """Fit K-means (Lloyd) to this rank's shard ``X`` (N_local, D) from ``centers_init`` (K, D).

    ``tol`` is the absolute centre-shift tolerance (sklearn's ``_tolerance``
    output, ``_kmeans.py:279-287``); 0 means "strict label convergence or
    max_iter".  ``group``: the process group whose ranks each hold one row shard
    (None = the default group when one is initialised); ``LOCAL`` forces a
    single-process fit of ``X`` alone.  ``engine`` lets tests substitute a CPU stand-in for the HIP engine.
    """
    if engine is None:
        from .engine import Engine
        engine = Engine(X.shape[1], centers_init.shape[0], X.dtype, max_iter=max_iter)
    prepare(engine, X, group, shard)
    x = exchange_for(engine, exchange, group)
    st, relocs = run(engine, centers_init, max_iter, tol, group, chunk, split, graph, x)
    labels, centers, inertia = finish(engine, group)
    ch, sh = engine.history(int(st["iter"]))
    layout = engine.layout_info()
    sl = getattr(engine, "_slab", None)
    layout["shard"] = "slab" if sl is not None else "rows"
    layout["exchange"] = ("peer" if x is not None else "collective") if _world(group)[0] > 1 else None
    if sl is not None:
        layout["slab_points"] = sl["n_slab"]
        layout["slab_axis"] = sl["axis"]
    return LloydResult(labels=labels, centers=centers, inertia=inertia, n_iter=int(st["iter"]),
                       strict=st["done"] == 1, stat_words_changed=ch, shift=sh, relocations=relocs, layout=layout)
