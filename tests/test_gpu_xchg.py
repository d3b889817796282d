"""GPU: the one-sided statistics exchange (csrc/pcm_xchg.hip, pcm_amd/xchg.py).

* linked exchanges of one process (the 1-GPU slab proxy's form): every rank
  pushes, then every rank waits and sums -- exact int64 sums for P = 2, 3, 8, 16,
  odd and large word counts, several rounds (both buffer parities, the epoch);
* the slab engines of a config-4-shaped split (P = 4 and 8) iterating through
  the exchange: centres bitwise equal to one engine on the whole cloud, and to
  the same split summed by torch;
* failure: a rank whose peer never pushes times out (bounded wait), its error
  word is set, the engine's status becomes done = 4 and ``lloyd.run`` raises.

Multi-process exchanges (IPC handles over gloo, ranks sharing cuda:0) run in
test_gpu_multirank.py and test_gpu_full_configs.py.
"""
import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import lloyd_ref as R  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pcm():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pcm_amd
    return pcm_amd


@pytest.mark.parametrize("P,words", [(2, 4097), (3, 1), (3, 4096), (8, 4097), (8, 20481), (16, 257)])
def test_linked_allreduce_exact(pcm, P, words):
    from pcm_amd import xchg
    xs = xchg.linked(words, P)
    g = torch.Generator(device="cuda").manual_seed(P * 1000 + words)
    for rnd in range(5):
        bufs = [torch.randint(-2**62, 2**62, (words,), dtype=torch.int64, device="cuda", generator=g)
                for _ in range(P)]
        want = sum(b.clone() for b in bufs)
        for r in range(P):
            xs[r].allreduce(bufs[r], 1)
        for r in range(P):
            xs[r].allreduce(bufs[r], 2)
        torch.cuda.synchronize()
        for r in range(P):
            assert torch.equal(bufs[r], want), (rnd, r)
    for x in xs:
        assert x.status() == {"err": 0, "epoch": 5}


def _slab_engines(X, K, P, iters):
    from pcm_amd import lloyd
    from pcm_amd.engine import Engine, shard_hist, shard_partition
    from pcm_amd.fixed import fixed_q
    N, D = X.shape
    lo, hi, maxabs = Engine(D, K, X.dtype, max_iter=1).bbox(X)
    q = fixed_q(maxabs)
    axis = int(np.argmax(hi - lo))
    inv = lloyd.SLAB_BINS / (hi[axis] - lo[axis])
    owner = lloyd.slab_owner(shard_hist(X, axis, lo[axis], inv, lloyd.SLAB_BINS).cpu().numpy(), P)
    Xp, rows, cnt = shard_partition(X, axis, lo[axis], inv, lloyd.SLAB_BINS, owner, P, 0)
    engines, off = [], 0
    for r in range(P):
        Xr, rr = Xp[off:off + int(cnt[r])], rows[off:off + int(cnt[r])]
        off += int(cnt[r])
        e = Engine(D, K, X.dtype, max_iter=iters)
        e.bbox(Xr)
        e.set_shard(rr, N)
        e.build(Xr, q, 0)
        engines.append(e)
    return engines


@pytest.mark.parametrize("P", [4, 8])
def test_slab_engines_through_peer_exchange(pcm, P):
    """P slab engines of one process iterate with the linked exchange between
    assign and update: centres bitwise equal to one engine fitting the whole cloud."""
    from pcm_amd import lloyd, xchg
    from pcm_amd.engine import Engine, synth_rows, synth_uniform
    N, K, D, iters = 4_000_000, 512, 3, 9
    X = synth_uniform(N, D, seed=3)
    C0 = synth_rows(R.init_indices(N, K), D, seed=3)
    engines = _slab_engines(X, K, P, iters)
    xs = xchg.linked(engines[0].stats.numel(), P)
    for e in engines:
        e.begin(C0, 0.0, iters)
    for _ in range(iters):
        for r, e in enumerate(engines):
            e.iter_local()
            e.exchange(xs[r], 1)
        for r, e in enumerate(engines):
            e.exchange(xs[r], 2)
            e.iter_global()
    sts = [e.status() for e in engines]
    assert all(s["iter"] == iters and not s["halt"] for s in sts), sts[0]
    C = [e.centers().cpu().numpy() for e in engines]
    one = Engine(D, K, torch.float32, max_iter=iters)
    lloyd.prepare(one, X, lloyd.LOCAL)
    one.begin(C0, 0.0, iters)
    one.iterate(iters)
    C1 = one.centers().cpu().numpy()
    for c in C:
        np.testing.assert_array_equal(c, C1)
    ch1, _ = one.history(iters)
    for e in engines:
        ch, _ = e.history(iters)
        np.testing.assert_array_equal(ch > 0, ch1 > 0)
    assert all(x.status()["epoch"] == iters for x in xs)


def test_exchange_timeout_is_bounded_and_fails_the_fit(pcm):
    """Rank 1 never pushes: rank 0's wait ends after the timeout, its error word
    and done = 4 gate the rest of the fit, lloyd.run raises."""
    from pcm_amd import _lib, lloyd, xchg
    from pcm_amd.engine import Engine, synth_rows, synth_uniform
    N, K, D = 200_000, 64, 3
    X = synth_uniform(N, D, seed=4)
    C0 = synth_rows(R.init_indices(N, K), D, seed=4)
    xs = xchg.linked(K * (D + 1) + 1, 2, timeout_s=0.5)
    e = Engine(D, K, torch.float32, max_iter=10)
    lloyd.prepare(e, X, lloyd.LOCAL)
    e.begin(C0, 0.0, 10)
    t0 = time.perf_counter()
    e.iter_local()
    e.exchange(xs[0], 3)
    e.iter_global()
    st = e.status()
    dt = time.perf_counter() - t0
    assert 0.4 < dt < 10.0
    assert st["done"] == lloyd.XCHG_FAILED and st["iter"] == 0
    assert xs[0].status()["err"] == 1
    # every later exchange and iteration is gated: nothing waits again
    t0 = time.perf_counter()
    e.iter_local()
    e.exchange(xs[0], 3)
    e.iter_global()
    e.status()
    assert time.perf_counter() - t0 < 0.4
    # lloyd.run through an exchange whose peer never pushes: raises at the first status read
    e2 = Engine(D, K, torch.float32, max_iter=10)
    lloyd.prepare(e2, X, lloyd.LOCAL)
    ys = xchg.linked(K * (D + 1) + 1, 2, timeout_s=0.3)
    with pytest.raises(_lib.PcmError, match="exchange timed out"):
        lloyd.run(e2, C0, 10, 0.0, lloyd.LOCAL, 4, True, False, ys[0])
