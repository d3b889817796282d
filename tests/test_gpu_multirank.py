"""GPU, world size 2: the row-sharded driver on the real HIP engine.

Two ranks share ``cuda:0`` (one box has one GPU; RCCL refuses two ranks on one
device, so the process group is gloo, which all-reduces the device tensors
through host staging).  Each rank fits its contiguous row shard with
``pcm_amd.lloyd_fit``: the global fixed-point exponents (MAX all-reduce), shard
offsets (all-gather), ``iter_local -> all_reduce(engine.stats) -> iter_global``
every iteration, and the empty-cluster relocation (every rank's device
relocation records all-gathered, then applied on every rank).  The result must
be bit-identical to the single-process GPU fit and to the oracle.
"""
import os
import socket
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import lloyd_ref as R  # noqa: E402

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, X, C0, max_iter, chunk, dtype, out_dir, shard, exchange):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    import pcm_amd
    n = X.shape[0]
    a, b = n * rank // world, n * (rank + 1) // world
    Xs = torch.from_numpy(np.ascontiguousarray(X[a:b])).to("cuda", dtype)
    res = pcm_amd.lloyd_fit(Xs, torch.from_numpy(C0).cuda(), max_iter=max_iter, tol=0.0, chunk=chunk, shard=shard,
                            exchange=exchange)
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), labels=res.labels.cpu().numpy(),
             centers=res.centers.cpu().numpy(), n_iter=res.n_iter, inertia=res.inertia, changed=res.stat_words_changed,
             relocs=res.relocations, shard=res.layout["shard"], slab_points=res.layout.get("slab_points", -1),
             exchange=str(res.layout["exchange"]))
    dist.barrier()
    dist.destroy_process_group()


def run_world(X, C0, max_iter, chunk, tmp_path, world=2, dtype=torch.float32, shard="auto", exchange="peer"):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, _free_port(), X, C0, max_iter, chunk, dtype, str(tmp_path), shard, exchange),
             nprocs=world, join=True)
    parts = [np.load(os.path.join(tmp_path, f"r{r}.npz")) for r in range(world)]
    if exchange != "auto":   # the exchange the fit actually used
        assert all(str(p["exchange"]) == exchange for p in parts)
    return parts


@pytest.fixture(scope="module")
def pcm():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pcm_amd
    return pcm_amd


def single(pcm, X, C0, max_iter, dtype=torch.float32):
    res = pcm.lloyd_fit(torch.from_numpy(X).to("cuda", dtype), torch.from_numpy(C0).cuda(), max_iter=max_iter,
                        tol=0.0)
    torch.cuda.synchronize()
    return res


def compare(parts, res1, ref):
    labels = np.concatenate([p["labels"] for p in parts])
    np.testing.assert_array_equal(labels, ref["labels"])
    np.testing.assert_array_equal(labels, res1.labels.cpu().numpy())
    for p in parts:
        np.testing.assert_array_equal(p["centers"], ref["centers"])
        np.testing.assert_array_equal(p["centers"], res1.centers.cpu().numpy())
        assert int(p["n_iter"]) == ref["n_iter"] == res1.n_iter
        np.testing.assert_array_equal(np.asarray(p["changed"]) > 0, np.asarray(ref["changed"]) > 0)
        assert float(p["inertia"]) == ref["inertia"] == res1.inertia   # exact limbs, all-reduced


@pytest.mark.parametrize("chunk,shard,exchange", [(1, "slab", "peer"), (5, "slab", "peer"), (5, "rows", "peer"),
                                                  (1, "slab", "collective"), (5, "rows", "collective")])
def test_two_ranks_hip_engine(pcm, tmp_path, chunk, shard, exchange):
    """Both statistics exchanges: the one-sided peer writes (IPC-mapped buffers of
    two processes sharing the GPU; with chunk 5 the iterations replay from a
    captured HIP graph, which the peer exchange allows over gloo) and gloo's
    all-reduce."""
    X = R.splitmix_uniform(300_000, 3, 41)
    C0 = X[R.init_indices(300_000, 256)]
    ref = R.lloyd_fit(X, C0, max_iter=12, fast=True)
    parts = run_world(X, C0, 12, chunk, tmp_path, shard=shard, exchange=exchange)
    assert all(str(p["shard"]) == shard for p in parts)
    compare(parts, single(pcm, X, C0, 12), ref)


def test_two_ranks_hip_engine_fp16_d4(pcm, tmp_path):
    X = R.splitmix_uniform(120_000, 4, 42).astype(np.float16).astype(np.float32)
    C0 = X[R.init_indices(120_000, 64)]
    ref = R.lloyd_fit(X, C0, max_iter=8, fast=True)
    parts = run_world(X, C0, 8, 3, tmp_path, dtype=torch.float16)
    compare(parts, single(pcm, X, C0, 8, torch.float16), ref)


@pytest.mark.parametrize("shard,exchange", [("slab", "peer"), ("rows", "peer"), ("slab", "collective")])
def test_two_ranks_hip_relocation_across_shards(pcm, tmp_path, shard, exchange):
    """Empty clusters whose farthest points sit on different ranks (slabs: the
    relocation tie-break uses the global rows carried by pcm_layout_shard)."""
    X = R.splitmix_uniform(40_000, 3, 43)
    X[1_000] = [3.0, 3.0, 3.0]           # rank 0's far outlier
    X[39_000] = [-2.0, 4.0, 1.0]         # rank 1's (farther)
    X[25_000] = [2.5, -1.5, 2.0]         # rank 1
    C0 = np.concatenate([X[:20], np.array([[50, 50, 50], [60, 60, 60], [70, 70, 70]], np.float32)])
    ref = R.lloyd_fit(X, C0, max_iter=20, fast=True)
    parts = run_world(X, C0, 20, 3, tmp_path, shard=shard, exchange=exchange)
    assert int(parts[0]["relocs"]) >= 1 and int(parts[1]["relocs"]) == int(parts[0]["relocs"])
    compare(parts, single(pcm, X, C0, 20), ref)


def test_three_ranks_hip_skewed_slabs(pcm, tmp_path):
    """Three ranks, skewed cloud with duplicates and far points: very unequal slab
    widths and a rank whose rows mostly move away; bit-identical to the oracle."""
    X = R.splitmix_uniform(90_000, 3, 44)
    X[:70_000] *= np.float32(0.01)
    X[70_000:72_000] = X[70_000]
    X[89_900:] += np.float32(40.0)
    C0 = X[R.init_indices(90_000, 64)]
    ref = R.lloyd_fit(X, C0, max_iter=10, fast=True)
    parts = run_world(X, C0, 10, 4, tmp_path, world=3)
    assert sum(int(p["slab_points"]) for p in parts) == 90_000
    compare(parts, single(pcm, X, C0, 10), ref)
