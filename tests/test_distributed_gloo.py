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


def _worker(rank, world, port, X, C0, max_iter, chunk, out_dir, local=False):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pcm_amd
    from cpu_engine import OracleEngine
    from pcm_amd.lloyd import LOCAL
    n = X.shape[0]
    a, b = (0, n) if local else (n * rank // world, n * (rank + 1) // world)
    eng = OracleEngine(X.shape[1], C0.shape[0], max_iter)
    res = pcm_amd.lloyd_fit(torch.from_numpy(X[a:b]), torch.from_numpy(C0), max_iter=max_iter, tol=0.0,
                            chunk=chunk, engine=eng, group=LOCAL if local else None)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), labels=res.labels.numpy(), centers=res.centers.numpy(),
             n_iter=res.n_iter, inertia=res.inertia, changed=res.changed, relocs=res.relocations)
    dist.barrier()
    dist.destroy_process_group()


def run_world(X, C0, max_iter, chunk, tmp_path, world=2, local=False):
    port = _free_port()
    mp.spawn(_worker, args=(world, port, X, C0, max_iter, chunk, str(tmp_path), local), nprocs=world, join=True)
    parts = [np.load(os.path.join(tmp_path, f"r{r}.npz")) for r in range(world)]
    return parts


@pytest.mark.parametrize("chunk", [1, 4])
def test_two_ranks_match_single_process(tmp_path, chunk):
    from oracle import lloyd_ref as R
    X = R.splitmix_uniform(6000, 3, 21)
    C0 = X[R.init_indices(6000, 24)]
    ref = R.lloyd_fit(X, C0, max_iter=15)
    parts = run_world(X, C0, 15, chunk, tmp_path)
    labels = np.concatenate([p["labels"] for p in parts])
    np.testing.assert_array_equal(labels, ref["labels"])
    for p in parts:
        np.testing.assert_array_equal(p["centers"], ref["centers"])
        assert int(p["n_iter"]) == ref["n_iter"]
        # the engine reports changed statistic words, the oracle changed labels: zero together
        np.testing.assert_array_equal(np.asarray(p["changed"]) > 0, np.asarray(ref["changed"]) > 0)
        assert float(p["inertia"]) == ref["inertia"]


def test_two_ranks_relocation(tmp_path):
    """Empty clusters whose farthest points live on different ranks."""
    from oracle import lloyd_ref as R
    X = R.splitmix_uniform(3000, 3, 22)
    X[100] = [3.0, 3.0, 3.0]        # far outliers: one per shard
    X[2900] = [-2.0, 4.0, 1.0]
    C0 = np.concatenate([X[:6], np.array([[50, 50, 50], [60, 60, 60], [70, 70, 70]], np.float32)])
    ref = R.lloyd_fit(X, C0, max_iter=20)
    parts = run_world(X, C0, 20, 3, tmp_path)
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
