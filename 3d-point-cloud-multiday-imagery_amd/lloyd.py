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

Multi-GPU: rank r owns a contiguous row shard; the only collective on the data
path is one SUM all-reduce of K*(D+1)+1 int64 per iteration (RCCL over xGMI with
the ``nccl`` backend).  Integer statistics make the result bit-identical for
any world size.
"""
from __future__ import annotations

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
    changed: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int64))
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


def prepare(engine, X, group=None):
    """Layout phase: global fixed-point exponents, shard offsets, cell sort."""
    import torch.distributed as dist
    world, rank = _world(group)
    _, _, maxabs = engine.bbox(X)
    n_local = int(X.shape[0])
    gidx0, n_total = 0, n_local
    if world > 1:
        dev = engine.stats_device
        m = torch.tensor(np.asarray(maxabs, dtype=np.float64), device=dev)
        dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
        maxabs = m.cpu().numpy()
        mine = torch.tensor([n_local], dtype=torch.int64, device=dev)
        parts = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
        dist.all_gather(parts, mine, group=group)
        counts = [int(p.item()) for p in parts]
        gidx0, n_total = sum(counts[:rank]), sum(counts)
    if n_total >= 2 ** 32:
        raise ValueError("at most 2**32 - 1 points in one fit")
    q = fixed_q(maxabs)
    engine.build(X, q, gidx0)
    return q, n_total


def _uses_graph(graph, world, group, split):
    import torch.distributed as dist
    if graph is not None:
        return bool(graph)
    if not (world > 1 or split) or not dist.is_initialized():
        return False
    try:
        return dist.get_backend(group) == "nccl"   # RCCL collectives can be captured; gloo's cannot
    except Exception:   # noqa: BLE001
        return False


def run(engine, C0, max_iter=300, tol=0.0, group=None, chunk=8, split=False, graph=None):
    """Iteration phase on a prepared engine.  Returns (status, relocations).

    One process: ``pcm_iterate`` (k_lloyd + fused k_step per iteration).  Several
    (or ``split``): ``iter_local`` (k_lloyd accumulating into the statistics
    buffer) -> all-reduce of the statistics (only when world > 1) ->
    ``iter_global`` (k_step on them).  With RCCL (``graph`` None = auto) a chunk
    of that sequence is captured once in a HIP graph and replayed: no host launch
    gaps between the kernels and the collective; the device control block gates
    iterations queued past convergence or a halt either way."""
    import torch
    import torch.distributed as dist
    world, _ = _world(group)
    engine.begin(C0, tol, max_iter)
    relocs = 0
    it = 0
    use_graph = _uses_graph(graph, world, group, split)
    captured = None

    def seq(n):
        for _ in range(n):
            engine.iter_local()
            if world > 1:
                dist.all_reduce(engine.stats, group=group)
            engine.iter_global()

    while True:
        n_enq = max(1, min(chunk, max_iter - it))
        if world == 1 and not split:
            engine.iterate(n_enq)
        elif use_graph and n_enq == chunk:
            if captured is None:
                try:
                    captured = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(captured):
                        seq(chunk)
                except Exception:   # noqa: BLE001 -- capture refused: eager launches
                    captured, use_graph = None, False
                    torch.cuda.synchronize()
                    seq(n_enq)
            if captured is not None:
                captured.replay()
        else:
            seq(n_enq)
        st = engine.status()
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
    st = engine.status()
    inertia = st["inertia"]
    if world > 1:   # exact integer limbs: the same inertia for any world size
        t = torch.tensor(list(st["inertia_limbs"]) + [st["inertia_overflow"]], dtype=torch.int64,
                         device=engine.stats_device)
        dist.all_reduce(t, group=group)
        v = [int(x) for x in t.cpu().tolist()]
        inertia = inertia_from_limbs(v[:3], st["inertia_scale"], v[3])
    return engine.labels(), engine.centers(), inertia


def lloyd_fit(X, centers_init, max_iter: int = 300, tol: float = 0.0, *, group=None, chunk: int = 8,
              engine=None, split: bool = False, graph=None) -> LloydResult:
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
    prepare(engine, X, group)
    st, relocs = run(engine, centers_init, max_iter, tol, group, chunk, split, graph)
    labels, centers, inertia = finish(engine, group)
    ch, sh = engine.history(int(st["iter"]))
    return LloydResult(labels=labels, centers=centers, inertia=inertia, n_iter=int(st["iter"]),
                       strict=st["done"] == 1, changed=ch, shift=sh, relocations=relocs,
                       layout=engine.layout_info())
