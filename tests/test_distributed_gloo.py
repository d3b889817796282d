"""CPU, world size 2 (gloo): the row-sharded multi-rank driver (pcm_amd.lloyd)
gives results bit-identical to a single-process fit.

The per-rank engine is the oracle-backed stand-in (tests/cpu_engine.py); what
is under test is the driver's distributed logic: global fixed-point exponents
(MAX all-reduce), shard offsets (all-gather), the per-iteration SUM all-reduce
of the integer statistics, device-gated chunked enqueue, and the empty-cluster
relocation (halt -> per-rank farthest points -> all-gather -> resume).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, X, C0, max_iter, chunk, out_dir, local=False, shard="auto", opts=None):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pcm_amd
    from cpu_engine import OracleEngine
    from pcm_amd import engine as E
    from pcm_amd import lloyd as L
    opts = opts or {}
    if "maxp" in opts:
        L.SLAB_MAXP = opts["maxp"]
    if "engine_cap" in opts:
        E.ENGINE_MAX_POINTS = opts["engine_cap"]
    n = X.shape[0]
    a, b = (0, n) if local else (n * rank // world, n * (rank + 1) // world)
    eng = OracleEngine(X.shape[1], C0.shape[0], max_iter)
    if opts.get("fail_build_rank") == rank:
        def bad_build(*args, **kw):
            raise RuntimeError("injected build failure")
        eng.build = bad_build
    if opts.get("fail_partition_rank") == rank:
        def bad_partition(*args, **kw):
            raise MemoryError("injected partition failure")
        eng.shard_partition = bad_partition
    try:
        res = pcm_amd.lloyd_fit(torch.from_numpy(X[a:b]), torch.from_numpy(C0), max_iter=max_iter, tol=0.0,
                                chunk=chunk, engine=eng, group=L.LOCAL if local else None, shard=shard)
    except Exception as exc:   # noqa: BLE001 -- the test inspects every rank's outcome
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), error=f"{type(exc).__name__}: {exc}")
        dist.destroy_process_group()
        return
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), labels=res.labels.numpy(), centers=res.centers.numpy(),
             n_iter=res.n_iter, inertia=res.inertia, changed=res.stat_words_changed, relocs=res.relocations,
             shard=res.layout.get("shard", "rows"), slab_points=res.layout.get("slab_points", -1))
    dist.barrier()
    dist.destroy_process_group()


def run_world(X, C0, max_iter, chunk, tmp_path, world=2, local=False, shard="auto", opts=None):
    port = _free_port()
    mp.spawn(_worker, args=(world, port, X, C0, max_iter, chunk, str(tmp_path), local, shard, opts), nprocs=world,
             join=True)
    parts = [np.load(os.path.join(tmp_path, f"r{r}.npz")) for r in range(world)]
    return parts


@pytest.mark.parametrize("chunk,shard", [(1, "slab"), (4, "slab"), (4, "rows")])
def test_two_ranks_match_single_process(tmp_path, chunk, shard):
    from oracle import lloyd_ref as R
    X = R.splitmix_uniform(6000, 3, 21)
    C0 = X[R.init_indices(6000, 24)]
    ref = R.lloyd_fit(X, C0, max_iter=15)
    parts = run_world(X, C0, 15, chunk, tmp_path, shard=shard)
    assert all(str(p["shard"]) == shard for p in parts)
    labels = np.concatenate([p["labels"] for p in parts])
    np.testing.assert_array_equal(labels, ref["labels"])
    for p in parts:
        np.testing.assert_array_equal(p["centers"], ref["centers"])
        assert int(p["n_iter"]) == ref["n_iter"]
        # the engine reports changed statistic words, the oracle changed labels: zero together
        np.testing.assert_array_equal(np.asarray(p["changed"]) > 0, np.asarray(ref["changed"]) > 0)
        assert float(p["inertia"]) == ref["inertia"]


@pytest.mark.parametrize("shard", ["slab", "rows"])
def test_two_ranks_relocation(tmp_path, shard):
    """Empty clusters whose farthest points live on different ranks."""
    from oracle import lloyd_ref as R
    X = R.splitmix_uniform(3000, 3, 22)
    X[100] = [3.0, 3.0, 3.0]        # far outliers: one per shard
    X[2900] = [-2.0, 4.0, 1.0]
    C0 = np.concatenate([X[:6], np.array([[50, 50, 50], [60, 60, 60], [70, 70, 70]], np.float32)])
    ref = R.lloyd_fit(X, C0, max_iter=20)
    parts = run_world(X, C0, 20, 3, tmp_path, shard=shard)
    labels = np.concatenate([p["labels"] for p in parts])
    assert int(parts[0]["relocs"]) >= 1
    np.testing.assert_array_equal(labels, ref["labels"])
    np.testing.assert_array_equal(parts[0]["centers"], ref["centers"])
    assert int(parts[1]["n_iter"]) == ref["n_iter"]


def test_local_group_under_default_group(tmp_path):
    """group=LOCAL (what the estimator and the plugin pass) fits the rank's whole
    X alone even when a default process group exists (counts and
    inertia were multiplied by the world size)."""
    from oracle import lloyd_ref as R
    X = R.splitmix_uniform(4000, 3, 23)
    C0 = X[R.init_indices(4000, 12)]
    ref = R.lloyd_fit(X, C0, max_iter=10)
    parts = run_world(X, C0, 10, 4, tmp_path, local=True)
    for p in parts:
        np.testing.assert_array_equal(p["labels"], ref["labels"])
        np.testing.assert_array_equal(p["centers"], ref["centers"])
        assert float(p["inertia"]) == ref["inertia"]


def test_slab_owner_equal_count_contiguous():
    from pcm_amd.lloyd import slab_owner
    rng = np.random.default_rng(0)
    h = rng.integers(0, 50, 1000)
    for world in (1, 2, 3, 8):
        own = slab_owner(h, world)
        assert own.dtype == np.uint8 and own.min() >= 0 and own.max() <= world - 1
        assert np.all(np.diff(own.astype(int)) >= 0)                       # contiguous slabs
        per = np.bincount(own, weights=h, minlength=world)
        assert np.all(np.abs(per - h.sum() / world) <= h.max())            # equal count up to one bin
    assert np.all(slab_owner(np.zeros(10, np.int64), 4) == 0)


def test_three_ranks_skewed_slabs(tmp_path):
    """Skewed cloud (most points in one corner, a few far away, duplicates): the
    equal-count slabs are very unequal in width, some bins are empty, a rank's
    row shard sends most of its rows elsewhere -- labels still come back in each
    rank's row order, bit-identical to the single-process fit."""
    from oracle import lloyd_ref as R
    X = R.splitmix_uniform(5000, 3, 24)
    X[:4000] *= np.float32(0.01)
    X[4000:4100] = X[4000]                    # exact duplicates
    X[4990:] += np.float32(40.0)
    C0 = X[R.init_indices(5000, 16)]
    ref = R.lloyd_fit(X, C0, max_iter=12)
    parts = run_world(X, C0, 12, 3, tmp_path, world=3)
    labels = np.concatenate([p["labels"] for p in parts])
    np.testing.assert_array_equal(labels, ref["labels"])
    assert sum(int(p["slab_points"]) for p in parts) == 5000
    for p in parts:
        np.testing.assert_array_equal(p["centers"], ref["centers"])
        assert int(p["n_iter"]) == ref["n_iter"]
        assert float(p["inertia"]) == ref["inertia"]


# ---------------------------------------------------------------- ADVICE r3 (slab limits, build failures)
def _check_fit(parts, ref):
    labels = np.concatenate([p["labels"] for p in parts])
    np.testing.assert_array_equal(labels, ref["labels"])
    for p in parts:
        np.testing.assert_array_equal(p["centers"], ref["centers"])
        assert int(p["n_iter"]) == ref["n_iter"]


def test_auto_falls_back_to_rows_past_the_slab_rank_limit(tmp_path):
    """More ranks than a slab partition addresses (PCM_SHARD_MAXP, lowered here
    to 1): shard='auto' keeps row shards, shard='slab' raises on every rank."""
    from oracle import lloyd_ref as R
    X = R.splitmix_uniform(4000, 3, 25)
    C0 = X[R.init_indices(4000, 10)]
    ref = R.lloyd_fit(X, C0, max_iter=8)
    parts = run_world(X, C0, 8, 4, tmp_path, opts={"maxp": 1})
    assert all(str(p["shard"]) == "rows" for p in parts)
    _check_fit(parts, ref)
    parts = run_world(X, C0, 8, 4, tmp_path, shard="slab", opts={"maxp": 1})
    assert all("ValueError" in str(p["error"]) for p in parts)


def test_oversized_slab_keeps_row_shards_on_every_rank(tmp_path):
    """A slab larger than one engine holds (the cap lowered to 2500 points; each
    of the two slabs would get 3000): every rank sees the same histogram and
    keeps its row shard, and the fit is unchanged."""
    from oracle import lloyd_ref as R
    X = R.splitmix_uniform(6000, 3, 26)
    C0 = X[R.init_indices(6000, 16)]
    ref = R.lloyd_fit(X, C0, max_iter=10)
    parts = run_world(X, C0, 10, 4, tmp_path, opts={"engine_cap": 2500})
    assert all(str(p["shard"]) == "rows" for p in parts)
    _check_fit(parts, ref)


def test_build_failure_on_one_rank_raises_on_every_rank(tmp_path):
    """engine.build failing on rank 1 only: both ranks raise (rank 0 learns it
    from the agreement all-reduce) instead of rank 0 blocking in the next
    collective."""
    from oracle import lloyd_ref as R
    X = R.splitmix_uniform(3000, 3, 27)
    C0 = X[R.init_indices(3000, 8)]
    for shard in ("slab", "rows"):
        parts = run_world(X, C0, 5, 4, tmp_path, shard=shard, opts={"fail_build_rank": 1})
        assert "injected build failure" in str(parts[1]["error"])
        assert "another rank" in str(parts[0]["error"])


def test_partition_failure_on_one_rank_raises_on_every_rank(tmp_path):
    """the slab partition (its workspace) failing on rank 1 only: both
    ranks raise before the all_to_all instead of rank 0 blocking in it."""
    from oracle import lloyd_ref as R
    X = R.splitmix_uniform(3000, 3, 28)
    C0 = X[R.init_indices(3000, 8)]
    parts = run_world(X, C0, 5, 4, tmp_path, shard="slab", opts={"fail_partition_rank": 1})
    assert "injected partition failure" in str(parts[1]["error"])
    assert "another rank" in str(parts[0]["error"])
