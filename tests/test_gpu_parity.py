"""GPU parity: the HIP engine (through the C ABI) vs the CPU oracle.

Bar (north_star): labels bit-exact; centres within 1e-5 relative of the
oracle -- here they are required to be bitwise equal, since the engine and the
oracle share the canonical arithmetic (exact integer sums, one fp64 division,
one rounding to fp32).  n_iter must match, and the per-iteration change
records must be zero at the same iterations.
"""
import glob
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import lloyd_ref as R  # noqa: E402

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def pcm():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pcm_amd
    from pcm_amd import _lib
    _lib.load()
    return pcm_amd


def gpu_fit(pcm, X, C0, max_iter, tol=0.0, dtype=torch.float32, chunk=8):
    Xt = torch.from_numpy(np.ascontiguousarray(X)).to("cuda", dtype)
    res = pcm.lloyd_fit(Xt, torch.from_numpy(np.ascontiguousarray(C0, dtype=np.float32)).cuda(),
                        max_iter=max_iter, tol=tol, chunk=chunk)
    torch.cuda.synchronize()
    return res


def assert_same(res, ref, where=""):
    lab = res.labels.cpu().numpy()
    cen = res.centers.cpu().numpy()
    assert res.n_iter == ref["n_iter"], f"{where} n_iter {res.n_iter} != {ref['n_iter']}"
    bad = np.flatnonzero(lab != ref["labels"])
    assert bad.size == 0, f"{where} {bad.size} labels differ, first rows {bad[:8]}"
    assert np.array_equal(cen, ref["centers"]), f"{where} centres differ: max {np.abs(cen - ref['centers']).max()}"
    # the engine counts changed statistic words, the oracle changed labels: zero together
    np.testing.assert_array_equal(res.stat_words_changed > 0, np.asarray(ref["changed"], dtype=np.int64) > 0)
    assert res.inertia == ref["inertia"]      # exact integer inertia: bitwise equal


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))), ids=os.path.basename)
def test_golden_fits(pcm, path):
    g = np.load(path)
    if "fit_labels" not in g:
        pytest.skip("step-only fixture")
    X, C0 = g["X"], g["C0"]
    ref = R.lloyd_fit(X, C0, max_iter=300, tol=0.0, fast=True)
    res = gpu_fit(pcm, X, C0, 300)
    assert_same(res, ref, os.path.basename(path))
    # and the sklearn golden itself (tolerance: sklearn sums in float32)
    np.testing.assert_array_equal(res.labels.cpu().numpy(), g["fit_labels"])
    assert res.n_iter == int(g["fit_n_iter"])
    scale = np.abs(X).max()
    np.testing.assert_allclose(res.centers.cpu().numpy(), g["fit_centers"], rtol=1e-5, atol=1e-5 * scale)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))), ids=os.path.basename)
def test_golden_steps(pcm, path):
    """One Lloyd step from each of sklearn's recorded centre sets: labels equal sklearn's."""
    g = np.load(path)
    X = g["X"]
    for t in range(g["labels"].shape[0]):
        res = gpu_fit(pcm, X, g["c_in"][t], 1)
        ref = R.lloyd_fit(X, g["c_in"][t], max_iter=1, fast=True)
        assert_same(res, ref, f"{os.path.basename(path)} step {t}")
        # labels of the first E-step = sklearn's labels for that step: re-run E only
        lab0 = R.assign(X, g["c_in"][t])
        np.testing.assert_array_equal(lab0, g["labels"][t])


CASES = [
    # n, k, d, dtype, max_iter, seed
    (100_000, 64, 3, "f32", 20, 1),
    (200_000, 1024, 3, "f32", 8, 2),
    (60_000, 16, 4, "f16", 12, 3),
    (30_000, 5, 2, "f32", 30, 4),
    (50_000, 300, 1, "f32", 10, 5),
    (1, 1, 3, "f32", 3, 6),
    (7, 7, 3, "f32", 3, 7),
    (4099, 4096, 3, "f32", 3, 8),
]


@pytest.mark.parametrize("n,k,d,dt,iters,seed", CASES)
def test_random_fit(pcm, n, k, d, dt, iters, seed):
    X = R.splitmix_uniform(n, d, seed)
    if dt == "f16":
        X = X.astype(np.float16).astype(np.float32)
    C0 = X[R.init_indices(n, k)]
    ref = R.lloyd_fit(X, C0, max_iter=iters, fast=True)
    res = gpu_fit(pcm, X, C0, iters, dtype=torch.float16 if dt == "f16" else torch.float32)
    assert_same(res, ref, f"n={n} k={k} d={d}")


def test_heightmap_like_cloud(pcm):
    """Anisotropic 2.5-D cloud in pixel units (z,y,x as plugin.py:191-192 emits)."""
    rng = np.random.default_rng(11)
    n = 150_000
    y = rng.integers(0, 1800, n).astype(np.float64)
    x = rng.integers(0, 2400, n).astype(np.float64)
    z = 10 * np.sin(x / 200) + 5 * np.cos(y / 150) + rng.normal(0, 0.5, n) + 30
    X = np.stack([z, y, x], axis=1).astype(np.float32)
    C0 = X[R.init_indices(n, 512)]
    ref = R.lloyd_fit(X, C0, max_iter=15, fast=True)
    res = gpu_fit(pcm, X, C0, 15)
    assert_same(res, ref, "heightmap")


def test_offset_cloud_and_negative(pcm):
    X = (R.splitmix_uniform(80_000, 3, 12) * np.float32(50) - np.float32(1.0e4)).astype(np.float32)
    C0 = X[R.init_indices(80_000, 200)]
    ref = R.lloyd_fit(X, C0, max_iter=10, fast=True)
    res = gpu_fit(pcm, X, C0, 10)
    assert_same(res, ref, "offset")


def test_ties_and_duplicates(pcm):
    base = np.random.default_rng(5).integers(0, 6, size=(5000, 3)).astype(np.float32)
    X = np.concatenate([base, base, base])
    C0 = np.concatenate([X[:10], X[:10]])     # every centre duplicated: exact ties everywhere
    ref = R.lloyd_fit(X, C0, max_iter=10, fast=True)
    res = gpu_fit(pcm, X, C0, 10)
    assert_same(res, ref, "ties")


def test_relocation_many_empty(pcm):
    X = R.splitmix_uniform(20_000, 3, 13)
    far = np.full((6, 3), 500.0, dtype=np.float32) + np.arange(6, dtype=np.float32)[:, None]
    C0 = np.concatenate([X[:10], far])        # 6 empty clusters on the first step
    ref = R.lloyd_fit(X, C0, max_iter=20, fast=True)
    res = gpu_fit(pcm, X, C0, 20, chunk=3)
    assert res.relocations >= 1
    assert_same(res, ref, "reloc")


def test_tol_convergence(pcm):
    X = R.splitmix_uniform(40_000, 3, 14)
    C0 = X[R.init_indices(40_000, 50)]
    ref = R.lloyd_fit(X, C0, max_iter=100, tol=1e-6, fast=True, history=True)
    res = gpu_fit(pcm, X, C0, 100, tol=1e-6)
    assert not res.strict
    assert_same(res, ref, "tol")
    # per-iteration centre shifts: the same fixed fp64 reduction tree on both sides
    np.testing.assert_array_equal(res.shift, np.array([h["shift"] for h in ref["history"]]))
    assert res.shift[-1] <= 1e-6 < res.shift[-2]


def test_bruteforce_operator(pcm):
    from pcm_amd.engine import assign_bruteforce
    X = R.splitmix_uniform(50_000, 3, 15)
    C = R.splitmix_uniform(700, 3, 16)
    q = R.fixed_q(X)
    stats = torch.zeros(700 * 4, dtype=torch.int64, device="cuda")
    lab = assign_bruteforce(torch.from_numpy(X).cuda(), torch.from_numpy(C).cuda(), q, stats)
    l2, s2, c2, _ = R.local_stats(X, C, np.full(len(X), -1, np.int32), q, fast=True)
    np.testing.assert_array_equal(lab.cpu().numpy(), l2)
    st = stats.cpu().numpy().reshape(700, 4)
    np.testing.assert_array_equal(st[:, 3], c2)
    np.testing.assert_array_equal(st[:, :3], s2)


def test_device_synth_matches_cpu(pcm):
    from pcm_amd.engine import synth_uniform
    a = synth_uniform(10_000, 3, seed=3, start=12345).cpu().numpy()
    np.testing.assert_array_equal(a, R.splitmix_uniform(10_000, 3, 3, start=12345))


def test_nonfinite_rejected(pcm):
    X = R.splitmix_uniform(1000, 3, 1)
    X[17, 1] = np.nan
    with pytest.raises(Exception, match="NaN"):
        gpu_fit(pcm, X, X[:4], 3)


def test_relocation_donor_emptied(pcm):
    X = np.array([[0.0, 0, 0], [0.1, 0, 0], [0.2, 0, 0], [100.0, 0, 0]], np.float32)
    C0 = np.array([[1000.0, 0, 0], [0.0, 0, 0], [90.0, 0, 0]], np.float32)
    ref = R.lloyd_fit(X, C0, max_iter=5)
    res = gpu_fit(pcm, X, C0, 5, chunk=1)
    assert res.relocations >= 1
    assert_same(res, ref, "donor")


def test_plugin_gpu_matches_oracle(pcm):
    from fake_pipeline import SyntheticPairExtractor
    plugin = pcm.HeightMapExtractor(base=SyntheticPairExtractor(n_pairs=3, shape=(90, 120)), n_clusters=64,
                                    max_iter=30, tol=0.0)
    layers = plugin.run("roi.kml")
    fused = [l for l in layers if "Fused" in l[1]["name"]]
    assert len(fused) == 2
    X = fused[1][0].astype(np.float32)
    C0 = X[R.init_indices(X.shape[0], 64)]
    ref = R.lloyd_fit(X, C0, max_iter=30, fast=True)
    np.testing.assert_array_equal(fused[1][1]["properties"]["cluster"], ref["labels"])
    np.testing.assert_array_equal(fused[0][0].astype(np.float32), ref["centers"])


@pytest.mark.parametrize("name", ["cfg1_n10k_k8", "n4096_k64", "empty_reloc", "d4_fp16"])
def test_split_call_sequence(pcm, name):
    """The multi-GPU call sequence (iter_local -> [all-reduce] -> iter_global: k_fold +
    k_step on `stats`) on one GPU gives the same fit as pcm_iterate and the oracle."""
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    X, C0 = g["X"], g["C0"]
    ref = R.lloyd_fit(X, C0, max_iter=300, tol=0.0, fast=True)
    dt = torch.float16 if X.dtype == np.float16 else torch.float32
    res = pcm.lloyd_fit(torch.from_numpy(np.ascontiguousarray(X)).to("cuda", dt),
                        torch.from_numpy(np.ascontiguousarray(C0, dtype=np.float32)).cuda(), max_iter=300,
                        tol=0.0, chunk=3, split=True)
    torch.cuda.synchronize()
    assert_same(res, ref, name)


def test_plugin_gpu_kmeanspp_init(pcm):
    """init='k-means++' (sklearn's default): GPU seeding + GPU Lloyd = oracle seeding + oracle Lloyd."""
    from fake_pipeline import SyntheticPairExtractor
    from oracle import kpp_ref as P
    plugin = pcm.HeightMapExtractor(base=SyntheticPairExtractor(n_pairs=2, shape=(80, 100)), n_clusters=32,
                                    max_iter=40, tol=0.0, init="k-means++", seed=5)
    layers = plugin.run("roi.kml")
    fused = [l for l in layers if "Fused" in l[1]["name"]]
    X = fused[1][0].astype(np.float32)
    C0, _ = P.kmeanspp(X, 32, 5)
    ref = R.lloyd_fit(X, C0, max_iter=40, fast=True)
    np.testing.assert_array_equal(fused[1][1]["properties"]["cluster"], ref["labels"])
    np.testing.assert_array_equal(fused[0][0].astype(np.float32), ref["centers"])


def test_unpruned_full_lists(pcm):
    """Extent >= 1e18 disables pruning: every cell scans all K centres (the
    FULL path, including the previous-iteration scan over the kept centres)."""
    X = (R.splitmix_uniform(6000, 3, 31).astype(np.float64) * 4e18 - 2e18).astype(np.float32)
    C0 = X[R.init_indices(6000, 24)]
    ref = R.lloyd_fit(X, C0, max_iter=25, tol=0.0, fast=True)
    res = gpu_fit(pcm, X, C0, 25)
    assert_same(res, ref, "unpruned")


def test_relocation_distance_ties_topm(pcm):
    """Radix-select relocation: many points at exactly the same (largest)
    distance -> the lowest global rows move first (distance desc, row asc)."""
    X = R.splitmix_uniform(200_000, 3, 33)
    far = np.array([7.0, 7.0, 7.0], np.float32)
    X[5_000:5_400] = far                       # 400 identical far points (equal keys' distance bits)
    X[150_000:150_200] = far
    C0 = np.concatenate([X[:40], np.full((12, 3), 900.0, np.float32) + np.arange(12, dtype=np.float32)[:, None]])
    ref = R.lloyd_fit(X, C0, max_iter=12, fast=True)
    res = gpu_fit(pcm, X, C0, 12, chunk=2)
    assert res.relocations >= 1
    assert_same(res, ref, "reloc ties")


@pytest.mark.parametrize("name", ["cfg1_n10k_k8", "empty_reloc"])
def test_split_sequence_graph_replay(pcm, name):
    """The multi-GPU call sequence captured in a HIP graph (a 1-rank RCCL group:
    k_lloyd -> all_reduce -> k_step per iteration, replayed per chunk) gives the
    oracle's fit, relocation included."""
    import socket
    import torch.distributed as dist
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    X, C0 = g["X"], g["C0"]
    ref = R.lloyd_fit(X, C0, max_iter=300, tol=0.0, fast=True)
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", world_size=1, rank=0,
                            device_id=torch.device("cuda", 0))
    try:
        res = pcm.lloyd_fit(torch.from_numpy(np.ascontiguousarray(X)).cuda(),
                            torch.from_numpy(np.ascontiguousarray(C0, dtype=np.float32)).cuda(), max_iter=300,
                            tol=0.0, chunk=4, split=True, graph=True)
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    assert_same(res, ref, name + " graph")


@pytest.mark.parametrize("slots", ["8", "16"])
def test_lane_slot_variants(pcm, slots, monkeypatch):
    """Both k_lloyd accumulation variants (8 lane slots + block-shared int64 LDS
    words for list positions >= 8, or 16 lane slots + global atomics beyond)
    on clouds whose lists are short (fine grid) and long (height-map cloud,
    K=512 over few cells: positions well past 8 and 16)."""
    monkeypatch.setenv("PCM_LSLOT_RT", slots)
    X = R.splitmix_uniform(300_000, 3, 21)
    C0 = X[R.init_indices(300_000, 24)]
    ref = R.lloyd_fit(X, C0, max_iter=6, fast=True)
    assert_same(gpu_fit(pcm, X, C0, 6), ref, f"short lists, {slots} slots")
    rng = np.random.default_rng(22)
    n = 120_000
    y = rng.integers(0, 600, n).astype(np.float64)
    x = rng.integers(0, 800, n).astype(np.float64)
    z = 10 * np.sin(x / 90) + rng.normal(0, 0.5, n) + 30
    X = np.stack([z, y, x], axis=1).astype(np.float32)
    C0 = X[R.init_indices(n, 512)]
    ref = R.lloyd_fit(X, C0, max_iter=6, fast=True)
    res = gpu_fit(pcm, X, C0, 6)
    assert_same(res, ref, f"long lists, {slots} slots")


def test_engine_reserve(pcm):
    """pcm_engine_reserve (engine setup) grows the point-sized buffers: fits on a
    reserved engine -- smaller, then larger clouds than reserved -- stay exact."""
    from pcm_amd.engine import Engine
    eng = Engine(3, 256, torch.float32, max_iter=8)
    eng.reserve(150_000)
    for n, seed in ((120_000, 21), (150_000, 22), (260_000, 23)):
        X = R.splitmix_uniform(n, 3, seed)
        C0 = X[R.init_indices(n, 256)]
        ref = R.lloyd_fit(X, C0, max_iter=8, fast=True)
        res = pcm.lloyd_fit(torch.from_numpy(X).cuda(), torch.from_numpy(C0).cuda(), max_iter=8, tol=0.0,
                            engine=eng)
        assert_same(res, ref, f"reserved engine n={n}")
    eng.reserve(400_000)            # invalidates the layout: iterating needs a new one
    from pcm_amd._lib import PcmError
    with pytest.raises(PcmError):
        eng.iterate(1)
    eng.close()


@pytest.mark.parametrize("fused", ["0", "1"])
def test_update_paths(pcm, fused, monkeypatch):
    """The centre update + list paths (k_upd1 + k_lists, or the fused k_updlists
    behind PCM_FUSED_UPD=1) against the oracle: list rebuilds and refreshes,
    an empty cluster (halt, relocation, resume) and tol convergence."""
    monkeypatch.setenv("PCM_FUSED_UPD", fused)
    X = R.splitmix_uniform(120_000, 3, 31)
    for k, iters, tol in ((1024, 12, 0.0), (700, 10, 0.0), (64, 40, 1e-6)):
        C0 = X[R.init_indices(X.shape[0], k)]
        ref = R.lloyd_fit(X, C0, max_iter=iters, tol=tol, fast=True)
        assert_same(gpu_fit(pcm, X, C0, iters, tol=tol), ref, f"fused={fused} k={k}")
    # relocation: duplicated initial centres leave clusters empty
    Xr = R.splitmix_uniform(50_000, 3, 32)
    C0 = Xr[R.init_indices(50_000, 200)].copy()
    C0[100:150] = C0[0]
    ref = R.lloyd_fit(Xr, C0, max_iter=15, fast=True)
    assert_same(gpu_fit(pcm, Xr, C0, 15), ref, f"fused={fused} relocation")


def test_update_paths_d4(pcm):
    """D = 4 update paths (k_upd1 for K <= 2048, else k_upd; k_coarse, then the
    256-thread k_lists<4, 2>) against the oracle: list rebuilds, fp16 points,
    an empty cluster."""
    fused = "-"
    X = R.splitmix_uniform(160_000, 4, 41).astype(np.float16).astype(np.float32)
    for k, iters in ((300, 10), (3000, 6)):
        C0 = X[R.init_indices(X.shape[0], k)]
        ref = R.lloyd_fit(X, C0, max_iter=iters, fast=True)
        assert_same(gpu_fit(pcm, X, C0, iters, dtype=torch.float16), ref, f"fused={fused} d4 k={k}")
    C0 = X[R.init_indices(X.shape[0], 120)].copy()
    C0[60:90] = C0[0]
    ref = R.lloyd_fit(X, C0, max_iter=8, fast=True)
    assert_same(gpu_fit(pcm, X, C0, 8, dtype=torch.float16), ref, f"fused={fused} d4 relocation")
    # K > 2048 (the multi-block k_upd with its release/acquire hand-off) through a relocation
    # (ADVICE r4): 40 duplicated centres leave 39 clusters empty at the first update
    C0 = X[R.init_indices(X.shape[0], 3000)].copy()
    C0[2000:2040] = C0[5]
    ref = R.lloyd_fit(X, C0, max_iter=6, fast=True)
    assert_same(gpu_fit(pcm, X, C0, 6, dtype=torch.float16), ref, f"fused={fused} d4 k=3000 relocation")
