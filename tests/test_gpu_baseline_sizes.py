"""GPU parity at the BASELINE.json configurations, full size.

The HIP engine (through the C ABI) against the bit-exact C restatement of the
oracle (oracle/lloyd_ref.c via ``lloyd_ref.lloyd_fit(fast=True)``, OpenMP on the
GPU box's host cores), on the same points:

* config 2: N=1M, K=64, D=3 fp32, 20 Lloyd iterations, full fit;
* config 3: N=100M, K=1024, D=3 fp32, 2 iterations (the headline workload; the
  device-generated cloud is copied to the host so both sides see identical
  bits) -- exercises the >2^26-point, multi-GB buffer addressing of k_lloyd;
* config 5 shard: N=62.5M (one of eight ranks' rows), K=4096, D=4 fp16,
  2 iterations -- the K > 2048 non-fused update path (k_global + k_cand) and
  long candidate lists.

Bar: labels bit-exact, centres bitwise equal, same n_iter, per-iteration
change records zero together, inertia bitwise equal (exact integer sum).
"""
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
    from pcm_amd import _lib
    _lib.load()
    return pcm_amd


def check(res, ref, where):
    lab = res.labels.cpu().numpy()
    cen = res.centers.cpu().numpy()
    assert res.n_iter == ref["n_iter"], f"{where}: n_iter {res.n_iter} != {ref['n_iter']}"
    bad = np.flatnonzero(lab != ref["labels"])
    assert bad.size == 0, f"{where}: {bad.size} labels differ, first rows {bad[:8]}"
    assert np.array_equal(cen, ref["centers"]), f"{where}: centres differ (max {np.abs(cen - ref['centers']).max()})"
    np.testing.assert_array_equal(res.stat_words_changed > 0, np.asarray(ref["changed"], dtype=np.int64) > 0)
    assert res.inertia == ref["inertia"]      # exact integer inertia: bitwise equal


def device_cloud(pcm, n, d, dtype=torch.float32):
    from pcm_amd.engine import synth_uniform
    X = synth_uniform(n, d, seed=0)
    return X if dtype == torch.float32 else X.to(dtype)


def test_config2_1m_k64_20_iters(pcm):
    n, k, d = 1_000_000, 64, 3
    X = device_cloud(pcm, n, d)
    rows = R.init_indices(n, k)
    C0 = X[torch.from_numpy(rows).cuda()].clone()
    res = pcm.lloyd_fit(X, C0, max_iter=20, tol=0.0)
    torch.cuda.synchronize()
    Xh = X.cpu().numpy()
    ref = R.lloyd_fit(Xh, C0.cpu().numpy(), max_iter=20, tol=0.0, fast=True)
    check(res, ref, "config 2")


def test_config3_100m_k1024_2_iters(pcm):
    n, k, d = 100_000_000, 1024, 3
    X = device_cloud(pcm, n, d)
    C0 = X[torch.from_numpy(R.init_indices(n, k)).cuda()].clone()
    res = pcm.lloyd_fit(X, C0, max_iter=2, tol=0.0)
    torch.cuda.synchronize()
    Xh = X.cpu().numpy()
    del X
    # the device generator is the CPU generator (spot-check a slice far into the cloud)
    np.testing.assert_array_equal(Xh[77_000_000:77_001_000], R.splitmix_uniform(1000, d, 0, start=77_000_000))
    ref = R.lloyd_fit(Xh, C0.cpu().numpy(), max_iter=2, tol=0.0, fast=True)
    check(res, ref, "config 3")
    assert res.layout["ncells"] > 1 and res.layout["ntiles"] >= res.layout["ncells"] // 2


def test_config5_shard_62m_k4096_d4_fp16(pcm):
    n, k, d = 62_500_000, 4096, 4
    Xh16 = device_cloud(pcm, n, d, torch.float16)
    C0 = Xh16[torch.from_numpy(R.init_indices(n, k)).cuda()].float().contiguous()
    res = pcm.lloyd_fit(Xh16, C0, max_iter=2, tol=0.0)
    torch.cuda.synchronize()
    Xh = Xh16.cpu().numpy().astype(np.float32)     # exact widening, as the kernels do
    del Xh16
    ref = R.lloyd_fit(Xh, C0.cpu().numpy(), max_iter=2, tol=0.0, fast=True)
    check(res, ref, "config 5 shard")
