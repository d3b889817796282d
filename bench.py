#!/usr/bin/env python3
"""Headline benchmark: Lloyd K-means point·iters/s at N=100M, K=1024, D=3 fp32.

BASELINE.json metric: "point·iters/sec at N=100M K=1024 D=3; achieved HBM GB/s
vs roofline" (config 3 on one GPU; config 4 = the same cloud row-sharded over N
GPUs, one process per GPU, RCCL all-reduce of the K*(D+1)+1 integer statistics
every iteration).

A step = one full Lloyd iteration over the whole cloud: candidate lists,
nearest-centroid assignment of every point, exact integer accumulation,
all-reduce (N>1), averaging/shift/convergence.  The cloud (counter-based
U[0,1)^3, generated on the device) is resident in HBM and laid out in cell
order before the timed region; that one-time layout is reported separately
as ``layout_ms`` (it is not repeated per iteration).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--n N] [--k K] [--d D]
  N > 1: either under torchrun (RANK/WORLD_SIZE set by the launcher), or plain
  ``python bench.py --gpus N``: the parent then starts N rank processes itself
  (before anything touches the GPU), one per GPU, and exits with their status.
  Each rank generates its contiguous row shard of the cloud on its GPU; the
  layout regroups the shards into spatial slabs (one all_to_all, in
  ``layout_ms``); every timed iteration all-reduces the K*(D+1)+1 statistics.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "point·iters/sec at N=100M K=1024 D=3; achieved HBM GB/s vs roofline"


def cpu_baseline(X, C, budget_s: float = 12.0) -> dict:
    """Oracle C restatement (OpenMP, all granted host cores) timed on whole
    config-3 iterations: the SAME N-point cloud (copied from the device) and
    initial centres, E-step + exact accumulation over all N points per pass
    (1-2 full-N iterations)."""
    from oracle import cref
    from oracle import lloyd_ref as R

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    n, d = X.shape
    k = C.shape[0]
    q = R.fixed_q(X)
    lab = np.full(n, -1, np.int32)
    reps, dt = 0, 0.0
    while reps < 2 and (reps == 0 or dt < budget_s / 2):
        t0 = time.perf_counter()
        lab, _, _, _ = cref.lloyd_stats(X, C, q, lab, nthreads=threads)
        dt += time.perf_counter() - t0
        reps += 1
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": n * reps / dt, "unit": "point·iters/s", "cores": threads, "kind": "port",
            "sample": f"{reps} full-N iteration(s) (E-step + exact accumulation over all {n} points of the "
                      f"bench cloud), K={k}, D={d}, oracle/lloyd_ref.c brute force "
                      f"(-O3 -ffp-contract=off, OpenMP {threads} threads, {cpu_model})"}


def numpy_baseline(X, C, budget_s: float = 6.0) -> dict:
    """The NumPy restatement (oracle/lloyd_ref.py local_stats: chunked direct-form
    distances, argmin, exact int64 accumulation -- the Python-level cost of the
    reference-style CPU path, BASELINE.md "CPU-baseline plan") timed on a leading
    subsample of the bench cloud, one E-step + accumulation pass over it, grown
    until the pass takes about budget_s / 4."""
    from oracle import lloyd_ref as R

    n_all, d = X.shape
    k = C.shape[0]
    q = R.fixed_q(X)
    m = min(n_all, 16384)
    while True:
        Xs = np.ascontiguousarray(X[:m])
        t0 = time.perf_counter()
        R.local_stats(Xs, C, np.full(m, -1, np.int32), q)
        dt = time.perf_counter() - t0
        if dt >= budget_s / 4 or m >= n_all:
            break
        m = min(n_all, m * 4)
    return {"value": m / dt, "unit": "point·iters/s", "cores": 1, "kind": "port",
            "sample": f"1 E-step + exact accumulation over the first {m} points of the bench cloud, K={k}, "
                      f"D={d}, oracle/lloyd_ref.py NumPy path (single process)"}


def cpu_fit_baseline(X, C, iters: int) -> dict:
    """Config 2 ('full run on both CPU and GPU'): the whole
    `iters`-iteration fit by oracle/lloyd_ref.c (OpenMP, all granted cores), plus
    its result for the GPU parity check."""
    from oracle import lloyd_ref as R

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    t0 = time.perf_counter()
    ref = R.lloyd_fit(X, C, max_iter=iters, tol=0.0, fast=True)
    dt = time.perf_counter() - t0
    n = X.shape[0]
    return {"value": n * ref["n_iter"] / dt, "unit": "point·iters/s", "cores": threads, "kind": "port",
            "fit_ms": dt * 1e3,
            "sample": f"the whole {ref['n_iter']}-iteration fit (+ final E-step) of all {n} points, K={C.shape[0]}, "
                      f"oracle/lloyd_ref.c brute force (OpenMP {threads} threads)"}, ref


def cloud_bench(H: int = 4000, W: int = 4000) -> dict:
    """Per-pair cloud assembly (plugin.py:147-192) of a synthetic HxW disparity:
    GPU (pcm_amd.assemble_cloud, host arrays in and out, like the plugin) vs the
    NumPy restatement (oracle/cloud_ref.py, the reference's own code path)."""
    import torch

    import pcm_amd
    from oracle import cloud_ref

    rng = np.random.default_rng(0)
    yy, xx = np.mgrid[0:H, 0:W]
    disp = -16.0 * (8 * np.sin(xx / 230.0) + 5 * np.cos(yy / 170.0) + rng.normal(0, 0.3, (H, W)))
    valid = rng.random((H, W)) > 0.1
    pcm_amd.assemble_cloud(disp[:64, :64], valid[:64, :64])      # warm-up (library, kernels)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pts, _, _ = pcm_amd.assemble_cloud(disp, valid)
    gpu_ms = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    ref, _, _ = cloud_ref.assemble(disp, valid)
    cpu_ms = (time.perf_counter() - t0) * 1e3
    assert pts.shape == ref.shape and np.array_equal(pts[:, 1:], ref[:, 1:])
    return {"pixels": H * W, "points": int(pts.shape[0]), "gpu_ms": gpu_ms, "cpu_numpy_ms": cpu_ms,
            "note": "host float64 disparity in, host (M,3) points out (PCIe included)"}


def stereo_bench(H: int = 4000, W: int = 4000, reps: int = 20) -> dict:
    """Stereo consistency gathers (row f3) on device-resident H x W inputs, HIP
    events around `reps` launches: algorithmic bytes = 24 B/px (photo: float64
    disparity + 2 float32 images + float64 out) and 33 B/px (L/R: 2 float64
    disparities + float64 out + uint8 mask)."""
    import torch

    import pcm_amd
    rng = np.random.default_rng(0)
    left = torch.from_numpy(rng.uniform(0, 255, (H, W)).astype(np.float32)).cuda()
    right = torch.from_numpy(rng.uniform(0, 255, (H, W)).astype(np.float32)).cuda()
    ld = torch.from_numpy(rng.uniform(-150, 60, (H, W))).cuda()
    rd = -ld + 0.5
    out = {}
    for name, fn, bpp in [("photoconsistency", lambda: pcm_amd.photoconsistency_map(left, right, ld, -144), 24),
                          ("lr_consistency", lambda: pcm_amd.left_right_consistency(ld, rd, -144, threshold=3), 33)]:
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        out[name] = {"ms": ms, "GBps": bpp * H * W / (ms * 1e-3) / 1e9, "bytes_per_px": bpp,
                     "frac_hbm": bpp * H * W / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS}
    out["pixels"] = H * W
    # the product path as disparity_map calls it (pipeline.use_gpu_gathers): host NumPy
    # arrays in and out -- upload, kernel, download -- beside the NumPy gathers it replaces
    # (oracle/consistency_ref.py, the reference's processing.py:94-115 / disparity.py:229-250)
    from oracle import consistency_ref
    hl, hr, hld, hrd = left.cpu().numpy(), right.cpu().numpy(), ld.cpu().numpy(), rd.cpu().numpy()
    host = {}
    for name, gpu_fn, cpu_fn in [
            ("photoconsistency", lambda: pcm_amd.photoconsistency_map(hl, hr, hld, -144),
             lambda: consistency_ref.photoconsistency_map(hl, hr, hld, -144)),
            ("lr_consistency", lambda: pcm_amd.left_right_consistency(hld, hrd, -144),
             lambda: consistency_ref.left_right_consistency(hld, hrd, -144))]:
        gpu_fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            g = gpu_fn()
        gpu_ms = (time.perf_counter() - t0) * 1e3 / 3
        t0 = time.perf_counter()
        c = cpu_fn()
        cpu_ms = (time.perf_counter() - t0) * 1e3
        assert np.array_equal(g, c)
        host[name] = {"gpu_host_io_ms": gpu_ms, "numpy_ms": cpu_ms, "speedup": cpu_ms / gpu_ms}
    out["host_numpy_in_out"] = host
    return out


def pmc_traffic(n, k, d, world):
    """HBM bytes per k_lloyd launch from a rocprofv3 --pmc summary of this same
    workload (tools/evidence.sh; FETCH_SIZE x2 for gfx950's halved wide-read
    count, + WRITE_SIZE, per MI355X_MICROARCH.md), or None."""
    path = os.environ.get("PCM_PMC_JSON") or os.path.join(ROOT, "profiles", "pmc_k_lloyd.json")
    if world != 1 or (n, k, d) != (100_000_000, 1024, 3) or not os.path.exists(path):
        return None, None
    with open(path) as f:
        pm = json.load(f)
    rd, wr = pm.get("hbm_read_bytes_corrected"), pm.get("hbm_write_bytes")
    if rd is None or wr is None:
        return None, None
    return rd + wr, os.path.relpath(path, ROOT)


FP32_PEAK_TFLOPS = 157.3       # MI355X vector FP32 (MI355X_MICROARCH.md; f32 MFMA runs at the same rate)


def compute_roofline(n: int, k: int, d: int, cand_mean: float, launch_ms: float) -> dict:
    """The assign kernel against the FP32 compute roofline (BASELINE.md "Reported per
    config"): (3D + 1) flop per point and candidate (D subtractions, D squares, D - 1
    additions, one compare) over the candidates actually scanned (the mean list
    length; the uniform cloud's cells hold equal point counts), and the brute-force
    equivalent over all K centres (what the pruning saves; above 1 means the pruned
    kernel beats a brute-force kernel running at peak)."""
    if launch_ms <= 0:
        return None
    fpc = 3 * d + 1
    t = launch_ms * 1e-3
    done = n * cand_mean * fpc / t / 1e12
    brute = n * k * fpc / t / 1e12
    return {"bound": "fp32 valu", "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s", "flop_per_point_candidate": fpc,
            "candidates_per_point": cand_mean, "achieved": done, "compute_frac": done / FP32_PEAK_TFLOPS,
            "bruteforce_equivalent": brute, "bruteforce_equivalent_frac": brute / FP32_PEAK_TFLOPS}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """``--gpus N`` without a launcher: start N rank processes of this script
    (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in their environment) and wait.  The
    parent never initialises the GPU.  Any rank failing terminates the others
    (by their own PIDs) and the parent returns the first failure's status."""
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:
                    q.terminate()
        time.sleep(0.05)
    return rc


def slab_proxy(args) -> dict:
    """Config 4 at P GPUs, rehearsed on one: the cloud is split into the P slabs
    lloyd.prepare would give P ranks (same histogram, owner table and stable
    partition), each slab gets its own engine (pcm_layout_shard: global rows,
    n_global), and every iteration runs iter_local on all P engines, sums their
    statistics (standing in for the RCCL all-reduce) and runs iter_global on all
    P.  HIP events around each engine's two launches give the per-rank cost of
    an iteration without the collective.  The centres after the run are checked
    against a single-engine fit of the whole cloud (bit-identical)."""
    import torch

    from pcm_amd import lloyd
    from pcm_amd.engine import ENGINE_MAX_POINTS, Engine, shard_hist, shard_partition, synth_rows, synth_uniform
    from pcm_amd.fixed import fixed_q

    torch.cuda.set_device(0)
    N, K, D, P = args.n, args.k, args.d, args.slab_of
    iters = args.warmup + args.steps
    pdt = torch.float16 if args.dtype == "f16" else torch.float32
    X = synth_uniform(N, D, seed=0).to(pdt)
    C0 = synth_rows(np.sort(np.random.default_rng(1).choice(N, K, replace=False)), D, seed=0).to(pdt).float()
    lo, hi, maxabs = Engine(D, K, pdt, max_iter=1).bbox(X)
    q = fixed_q(maxabs)
    axis = int(np.argmax(hi - lo))
    inv = lloyd.SLAB_BINS / (hi[axis] - lo[axis])
    owner = lloyd.slab_owner(shard_hist(X, axis, lo[axis], inv, lloyd.SLAB_BINS).cpu().numpy(), P)
    Xp, rows, cnt = shard_partition(X, axis, lo[axis], inv, lloyd.SLAB_BINS, owner, P, 0)
    engines, off = [], 0
    for r in range(P):
        Xr, rr = Xp[off:off + int(cnt[r])], rows[off:off + int(cnt[r])]
        off += int(cnt[r])
        e = Engine(D, K, pdt, max_iter=iters + 4)
        e.bbox(Xr)
        e.set_shard(rr, N)
        e.build(Xr, q, 0)
        e.begin(C0, 0.0, iters + 4)
        engines.append(e)
    del Xp
    # one event set per timed step, read after the last one: the queue never runs
    # dry between steps (a per-step synchronize let the first engine's start event
    # fire before the host had submitted its kernel -- the round-3 "first-engine
    # artefact", ~8 us)
    ev = [[[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(P)] for _ in range(args.steps)]
    t_assign = np.zeros(P)
    t_step = np.zeros(P)
    peer = args.exchange != "collective"
    xs = None
    if peer:
        # the peer exchange between the P engines (linked receive buffers of one
        # process): each "rank" pushes after its assign and waits + sums before its
        # update, so both halves of the exchange are inside its timed spans
        from pcm_amd import xchg
        xs = xchg.linked(engines[0].stats.numel(), P)

    def step(evs):
        for r, e in enumerate(engines):
            if evs:
                evs[r][0].record()
            e.iter_local()
            if peer:
                e.exchange(xs[r], 1)
            if evs:
                evs[r][1].record()
        if not peer:
            total = engines[0].stats.clone()
            for e in engines[1:]:
                total += e.stats
            for e in engines:
                e.stats.copy_(total)
        for r, e in enumerate(engines):
            if evs:
                evs[r][2].record()
            if peer:
                e.exchange(xs[r], 2)
            e.iter_global()
            if evs:
                evs[r][3].record()

    for _ in range(args.warmup):
        step(None)
    torch.cuda.synchronize()
    for k in range(args.steps):
        step(ev[k])
    torch.cuda.synchronize()
    for k in range(args.steps):
        for r in range(P):
            t_assign[r] += ev[k][r][0].elapsed_time(ev[k][r][1])
            t_step[r] += ev[k][r][2].elapsed_time(ev[k][r][3])
    st = [e.status() for e in engines]
    if any(s["halt"] or s["iter"] != iters for s in st):
        raise SystemExit(f"slab proxy: iterations did not all run: {st[0]}")
    C_slab = engines[0].centers().cpu().numpy()
    ok = all(np.array_equal(C_slab, e.centers().cpu().numpy()) for e in engines)
    info = [dict(e.layout_info(), points=int(e.n), kernel=e.assign_kernel(), **e.candidate_stats()) for e in engines]
    del engines
    if N <= ENGINE_MAX_POINTS and os.environ.get("PCM_PROXY_NOCHECK") != "1":   # (=1: kernel traces of the proxy alone)
        one = Engine(D, K, pdt, max_iter=iters + 4)
        lloyd.prepare(one, X, lloyd.LOCAL)
        one.begin(C0, 0.0, iters + 4)
        one.iterate(iters)
        bitwise = bool(ok and np.array_equal(C_slab, one.centers().cpu().numpy()))
    else:       # one engine cannot hold the whole cloud: the P slab engines agreeing is the check left
        bitwise = None
    a_ms, s_ms = t_assign / args.steps, t_step / args.steps
    per_rank = (a_ms + s_ms) * 1e3
    what = ("peer exchange included: push after the assign, wait + sum before the update, linked buffers of one "
            "process (the xGMI hop itself not modelled)") if peer else "all-reduce excluded"
    return {"metric": f"per-rank Lloyd iteration cost at P GPUs (1-GPU slab proxy, {what})",
            "value": float(per_rank.max()), "unit": "us/iter (max over ranks)", "higher_is_better": False,
            "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "slab_of": P,
            "config": {"workload": f"{'config 5' if args.dtype == 'f16' else 'config 4'} split {P} ways: N={N} "
                                   f"K={K} D={D} {args.dtype}, slabs of axis {axis}"},
            "per_rank_us": {"assign": (a_ms * 1e3).round(2).tolist(), "step": (s_ms * 1e3).round(2).tolist(),
                            "total": per_rank.round(2).tolist()},
            "exchange": "peer (linked)" if peer else "host-summed (all-reduce emulated)",
            "slabs": info, "centres_bitwise_equal_single_engine": bitwise,
            "slab_engines_agree": bool(ok)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--d", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--fit", "--kpp", dest="fit", action="store_true",
                    help="time GPU k-means++ seeding (K centres) of the bench cloud (the default at N = 1 on "
                         "the headline config since round 5; kept for older command lines)")
    ap.add_argument("--no-kpp", action="store_true", help="skip the k-means++ timing")
    ap.add_argument("--fit-iters", type=int, default=20, help="iterations of the timed whole fit (0: skip)")
    ap.add_argument("--split", action="store_true",
                    help="one GPU through the multi-GPU call sequence (nccl group of 1; calibration)")
    ap.add_argument("--no-graph", dest="graph", action="store_false",
                    help="launch the timed iterations eagerly instead of replaying one captured HIP graph of "
                         "them (k_lloyd [+ RCCL all-reduce at N > 1] + k_step per iteration)")
    ap.add_argument("--no-events", action="store_true", help="calibration: no per-kernel HIP events")
    ap.add_argument("--stereo", action="store_true", help="also time the stereo consistency gathers (4000x4000)")
    ap.add_argument("--cloud", action="store_true",
                    help="also time the per-pair cloud assembly (4000x4000 disparity) on GPU and CPU")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend at N > 1 (nccl = RCCL over xGMI; gloo: rehearsal of N ranks sharing "
                         "one GPU, eager launches, host-staged collectives -- not a measurement)")
    ap.add_argument("--shard", default="slab", choices=["slab", "rows"],
                    help="N > 1: regroup the row shards into spatial slabs at layout time (default) or keep rows")
    ap.add_argument("--slab-of", type=int, default=0, metavar="P",
                    help="1-GPU proxy of config 4 at P GPUs: the P slab engines of lloyd.prepare's split run on this "
                         "GPU, their statistics summed between the kernels (the all-reduce, emulated); per-rank "
                         "k_lloyd1 + k_step times from HIP events (the per-rank iteration cost, RCCL excluded)")
    ap.add_argument("--exchange", default="auto", choices=["auto", "peer", "collective"],
                    help="N > 1: how the ranks sum the statistics every iteration -- peer (one-sided writes into the "
                         "peers' memory, pcm_amd/xchg.py), collective (torch.distributed all_reduce: RCCL) or auto "
                         "(peer when its setup and self-test pass on every rank); --slab-of P: peer (default) or "
                         "collective (the statistics summed by torch between the kernels)")
    ap.add_argument("--dtype", default="f32", choices=["f32", "f16"],
                    help="point dtype (f16: config 5's storage; the arithmetic stays canonical fp32)")
    ap.add_argument("--clustered", type=int, default=0, metavar="C",
                    help="degenerate-cloud check: C tight Gaussian clusters (sigma 0.004) + 1%% uniform background "
                         "instead of the uniform cloud (pruning stress: FULL candidate lists, long lists)")
    ap.add_argument("--config", type=int, default=0, choices=[0, 2, 3, 4, 5],
                    help="BASELINE.json config preset: 2 = N=1M K=64 D=3 f32, 20 timed iterations, GPU and CPU "
                         "whole 20-iteration fits with a bitwise parity check; 3/4 = the defaults (4: run with "
                         "--gpus N); 5 = N=500M K=4096 D=4 f16 (needs >= 2 GPUs: 2^28 points per engine)")
    ap.add_argument("--dry-launch", action="store_true",
                    help="launcher test: each rank prints its RANK/WORLD_SIZE as JSON and exits before any GPU call")
    args = ap.parse_args()
    if args.config == 2:
        args.n, args.k, args.d, args.dtype, args.steps = 1_000_000, 64, 3, "f32", 20
    elif args.config == 5:
        args.n, args.k, args.d, args.dtype = 500_000_000, 4096, 4, "f16"

    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and env_world is None:
        raise SystemExit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        raise SystemExit(2)
    if args.dry_launch:
        print(json.dumps({"rank": rank, "local_rank": local, "world_size": world,
                          "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}"}), flush=True)
        return

    import torch
    import torch.distributed as dist

    if args.slab_of > 1:
        if world != 1:
            raise SystemExit("--slab-of is a single-process proxy")
        print(json.dumps(slab_proxy(args)), flush=True)
        return

    ndev = torch.cuda.device_count()
    if args.backend == "nccl" and world > ndev:
        print(f"bench.py: {world} ranks but {ndev} visible GPUs (RCCL needs one GPU per rank)", file=sys.stderr)
        raise SystemExit(2)
    dev_index = local % max(1, ndev)
    torch.cuda.set_device(dev_index)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group("gloo")
        if dist.get_world_size() != args.gpus:
            print(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}", file=sys.stderr)
            raise SystemExit(2)
    elif args.split:
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", world_size=1, rank=0,
                                device_id=torch.device("cuda", dev_index))
    multi = world > 1 or args.split
    if world > 1 and args.backend == "gloo" and args.exchange == "collective":
        args.graph = False          # gloo collectives cannot be captured

    import pcm_amd
    from pcm_amd import lloyd
    from pcm_amd.engine import Engine, synth_rows, synth_uniform

    N, K, D = args.n, args.k, args.d
    lo_row = N * rank // world
    hi_row = N * (rank + 1) // world
    pdt = torch.float16 if args.dtype == "f16" else torch.float32
    X = synth_uniform(hi_row - lo_row, D, seed=0, start=lo_row)
    init_rows = np.sort(np.random.default_rng(1).choice(N, K, replace=False))
    C0 = synth_rows(init_rows, D, seed=0)
    if args.clustered > 0:
        # C tight clusters: each row's cluster and offset from the counter-based uniforms
        # (torch elementwise plumbing on the device), 1 % of the rows stay uniform background
        g = torch.Generator(device="cuda").manual_seed(5)
        centres = torch.rand((args.clustered, D), generator=g, device="cuda")
        cid = (X[:, 0] * args.clustered).long().clamp_(0, args.clustered - 1)
        noise = torch.randn(X.shape, generator=g, device="cuda") * 0.004
        keep = (X[:, 1] < 0.01).unsqueeze(1)
        X = torch.where(keep, X, centres[cid] + noise).contiguous()
        C0 = X[torch.as_tensor(init_rows - lo_row if world == 1 else init_rows % X.shape[0], device="cuda")].contiguous()
    if pdt == torch.float16:      # config 5 storage: the points and the initial centres rounded to fp16
        X = X.to(pdt).contiguous()
        C0 = C0.to(pdt).float()
    total_iters = args.warmup + args.steps
    max_iter = 2 * total_iters + 16      # timed steps + the eager event pass of as many
    group = None
    eng = Engine(D, K, pdt, max_iter=max_iter)
    # engine setup: the point-sized device buffers grown (and the fresh VRAM mapped)
    # before the timed layout -- a spatial slab holds ~N/world points, 1/8 headroom
    t0 = time.perf_counter()
    eng.reserve(int(X.shape[0] * (1.125 if world > 1 and args.shard == "slab" else 1.0)))
    torch.cuda.synchronize()
    reserve_ms = (time.perf_counter() - t0) * 1e3
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    lloyd.prepare(eng, X, group, args.shard)
    torch.cuda.synchronize()
    layout_ms = (time.perf_counter() - t0) * 1e3
    xch = None
    if world > 1:
        # the per-iteration statistics sum: the peer exchange (verified on every rank) or the collective
        xch = lloyd.exchange_for(eng, args.exchange)
    eng.begin(C0, 0.0, max_iter)

    ar_events = []

    def iterate(n, record=False):
        if not multi:
            eng.iterate(n)
        else:
            for _ in range(n):
                eng.iter_local()
                if record:   # HIP events around the exchange on the launch stream (RCCL's stream joins it)
                    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    ev[0].record()
                if xch is not None:
                    eng.exchange(xch)
                else:
                    dist.all_reduce(eng.stats)
                if record:
                    ev[1].record()
                    ar_events.append(ev)
                eng.iter_global()

    iterate(args.warmup)
    torch.cuda.synchronize()
    st = eng.status()
    if st["halt"] or st["done"]:
        raise SystemExit(f"fit stopped during warm-up: {st}")
    graph = None
    timing = "events in the timed region"
    if args.graph:
        # the timed steps as one captured HIP graph -- multi-GPU: k_lloyd, RCCL
        # all-reduce, k_step per iteration; one GPU: k_lloyd + k_step per iteration.
        # Device-side gating keeps the captured iterations exact; eager launches
        # if capture is refused.  (HIP event records captured in a graph cannot be
        # read back with hipEventElapsedTime here, so the per-kernel durations of
        # the roofline come from an eager pass of the same kernels right after.)
        try:
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                iterate(args.steps)
            torch.cuda.synchronize()
        except Exception as exc:   # noqa: BLE001 -- measurement fallback, reported in the JSON
            graph = None
            args.graph_error = repr(exc)[:200]
            torch.cuda.synchronize()
        # every rank replays (or every rank launches eagerly): collective sequences stay aligned
        if not lloyd.agree(graph is not None, world, None, eng.stats_device):
            graph = None
            args.graph_error = getattr(args, "graph_error", None) or "capture failed on another rank"
        # capture recorded the launches without running them
        if eng.status()["iter"] != args.warmup:
            raise SystemExit("graph capture executed iterations")
    if graph is None and not args.no_events and world == 1:
        # per-kernel HIP events inside the timed region (eager launches)
        eng.timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if graph is not None:
        graph.replay()
    else:
        iterate(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if not args.no_events and world == 1 and graph is None:
        tm = eng.timing_read()
    elif not args.no_events:
        # eager pass of the same kernels right after the timed graph replay (and, at
        # N > 1, where events inside the timed region would cost ~15 % of a shard's step)
        eng.timing(True)
        iterate(args.steps, record=multi)
        tm = eng.timing_read()
        timing = "HIP events on an eager pass of the same kernels right after the timed graph replay"
    else:
        tm = {"assign_ms": 0.0, "tail_ms": 0.0}
    st = eng.status()
    if st["iter"] < total_iters or st["halt"]:
        raise SystemExit(f"timed iterations did not all run: {st}")
    cand = eng.candidate_stats()
    cand["list_rebuilds"] = st.get("list_rebuilds")
    cand["iterations"] = st["iter"]
    info = eng.layout_info()
    torch.cuda.synchronize()
    allreduce_ms = (sum(a.elapsed_time(b) for a, b in ar_events) / len(ar_events)) if ar_events else None
    per_rank = None
    if world > 1:
        # per-rank breakdown of one iteration (eager event pass): assign, update, lists, the
        # all-reduce (its events include waiting for the slowest rank), the slab size
        mine = torch.tensor([dt, tm["assign_ms"], tm["tail_ms"], tm.get("candidates_ms", 0.0),
                             allreduce_ms if allreduce_ms is not None else -1.0, float(eng.n)],
                            dtype=torch.float64, device="cuda" if args.backend == "nccl" else "cpu")
        every = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
        every = torch.stack(every).cpu().numpy()
        dt, assign_ms = float(every[:, 0].max()), float(every[:, 1].max())
        per_rank = {"assign": every[:, 1].round(5).tolist(), "update": every[:, 2].round(5).tolist(),
                    "tile_lists": every[:, 3].round(5).tolist(),
                    "exchange" if xch is not None else "allreduce":
                        every[:, 4].round(5).tolist() if allreduce_ms is not None else None,
                    "points": every[:, 5].astype(np.int64).tolist(),
                    "wall_ms_per_step": (every[:, 0] * 1e3 / args.steps).round(5).tolist()}
        # every rank must hold the same centres after the run (they are computed from the
        # summed statistics): a cheap end-to-end check of the exchange at this world size
        ch = eng.centers().reshape(-1).view(torch.int32).to(torch.int64)
        digest = torch.stack([ch.sum(), (ch * torch.arange(1, ch.numel() + 1, device=ch.device)).sum()])
        digest = digest.to("cuda" if args.backend == "nccl" else "cpu")
        dg = [torch.zeros_like(digest) for _ in range(world)]
        dist.all_gather(dg, digest)
        per_rank["centres_agree"] = bool(all(torch.equal(d, dg[0]) for d in dg))
    else:
        assign_ms = tm["assign_ms"]
    launch_ms, b2b_ms = assign_ms, None
    if world == 1 and not args.no_events:
        # reported beside the roofline, not used by it: ONE HIP event pair around
        # `steps` back-to-back assign launches on the final layout, lists and centres
        # (no per-launch events, no k_step between them; the statistics they add are
        # discarded -- nothing iterates this engine afterwards).  They run ~10 % faster
        # than the same kernel inside the timed replay (rocprof, profiles/r4g_*) because
        # the kernel gets cheaper as the fit settles (profiles/r4i_*), so the roofline
        # keeps the eager-pass events, the closest to the timed region.
        b2b_ms = eng.time_assign(args.steps)

    fit = kpp_ms = None
    if args.fit_iters > 0 and world == 1:
        # whole fits (layout + iterations + final E-step + labels in the caller's
        # row order): a fresh engine (device buffers allocated) and the same
        # engine fitting again (persistent buffers reused)
        fit = {"iters": args.fit_iters}
        eng2 = Engine(D, K, pdt, max_iter=args.fit_iters)
        for key in ("cold_ms", "warm_ms"):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = pcm_amd.lloyd_fit(X, C0, max_iter=args.fit_iters, tol=0.0, engine=eng2)
            torch.cuda.synchronize()
            fit[key] = (time.perf_counter() - t0) * 1e3
            if res.n_iter != args.fit_iters:
                raise SystemExit(f"fit stopped after {res.n_iter} iterations")
            del res
        fit["pt_iters_per_s"] = N * args.fit_iters / (fit["warm_ms"] * 1e-3)
        del eng2
    kpp_cold_ms = None
    headline = (args.n, args.k, args.d, args.dtype) == (100_000_000, 1024, 3, "f32") and not args.split
    if (args.fit or headline) and not args.no_kpp and world == 1:
        # twice: the first call of the process allocates the workspace (torch's
        # caching allocator keeps it); the reference's call site seeds n_init=10
        # times (core.py:227-228), so the second call is the steady cost
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pcm_amd.kmeans_plusplus(X, K, random_state=0)
            torch.cuda.synchronize()
            if rep == 0:
                kpp_cold_ms = (time.perf_counter() - t0) * 1e3
            else:
                kpp_ms = (time.perf_counter() - t0) * 1e3

    if rank == 0:
        n_local = int(eng.n)      # points this rank's engine holds (its slab at N > 1)
        shape = (N, K, D, args.dtype)
        named = {(100_000_000, 1024, 3, "f32"): "config 3" if world == 1 else "config 4",
                 (500_000_000, 4096, 4, "f16"): "config 5", (1_000_000, 64, 3, "f32"): "config 2"}.get(shape)
        where = "1 GPU" if world == 1 else (f"{world} GPUs, {'spatial slabs' if args.shard == 'slab' else 'row shards'}, "
                                            f"all-reduce every iteration")
        workload = f"Lloyd K-means iteration, N={N} K={K} D={D} {args.dtype} ({(named + ', ') if named else ''}{where})"
        # the iteration kernel streams only the points (labels are recomputed, not stored):
        # 8 B/pt in compressed tiles (exact fp32 rebuilt from per-tile bases + delta bits),
        # D*4 B/pt elsewhere -- the roofline uses those streamed bytes, measured per layout
        # (roofline basis: SURVEY.md §8d's algorithmic bytes = one D*4-byte row per point per
        # iteration; the stream actually moved is reported beside it and by the PMC traffic)
        sb = eng.stream_bytes()
        stream_bytes = sb["bytes"]
        bytes_pt = D * (2 if pdt == torch.float16 else 4)
        achieved = bytes_pt * n_local / (launch_ms * 1e-3) / 1e9 if launch_ms > 0 else 0.0
        traffic, traffic_src = pmc_traffic(N, K, D, world)
        value = N * args.steps / dt
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "point·iters/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic: counter-based U[0,1)^3 cloud generated on device (splitmix64), init = rows "
                    "sorted(default_rng(1).choice(N, K))",
            "config": {"workload": workload + (f"; CLUSTERED cloud ({args.clustered} clusters), not config 3"
                                                if args.clustered else ""),
                       "n_points": N, "k": K, "d": D,
                       "parallelism": f"dp{world} ({'spatial slabs' if args.shard == 'slab' else 'row shards'})"
                                      if world > 1 else "single GPU",
                       "backend": (args.backend if world > 1 else ("nccl (group of 1)" if multi else None)),
                       "exchange": (("peer (one-sided writes into the peers' memory)" if xch is not None
                                     else "collective all_reduce") if world > 1 else None),
                       "launch": "hip-graph" if graph is not None else "eager",
                       "cells": info["ncells"], "tiles": info["ntiles"], "grid": info["grid"],
                       "rank0_points": n_local},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": eng.assign_kernel(),
                         "algorithmic_bytes_per_point": bytes_pt,
                         "stream_bytes_per_launch": stream_bytes, "compressed_points": sb["compressed_points"],
                         "stream_GBps": stream_bytes / (launch_ms * 1e-3) / 1e9 if launch_ms > 0 else 0.0,
                         "avg_launch_ms": launch_ms, "avg_launch_ms_back_to_back": b2b_ms,
                         "timing": timing + ("" if world == 1 else " (max over ranks)"),
                         "compute": compute_roofline(n_local, K, D, cand.get("mean", 0.0), launch_ms)},
            "breakdown_ms_per_iter": {"assign": assign_ms, "update": tm["tail_ms"],
                                      "tile_lists": tm.get("candidates_ms", 0.0),
                                      **({("exchange" if xch is not None else "allreduce"): allreduce_ms}
                                         if allreduce_ms is not None else {}),
                                      **({"per_rank": per_rank} if per_rank is not None else {})},
            "candidates": cand,
            "layout_ms": layout_ms,
            "reserve_ms": reserve_ms,   # engine setup (Engine.reserve), before the timed layout
        }
        if getattr(args, "graph_error", None):
            out["graph_error"] = args.graph_error
        if fit is not None:
            # whole-fit throughput (layout + iterations + final E-step + unpermute)
            out[f"fit_{fit['iters']}_iters_ms"] = fit["warm_ms"]
            out["fit"] = fit
        if args.cloud:
            out["cloud_assembly"] = cloud_bench()
        if args.stereo:
            out["stereo_gathers"] = stereo_bench()
        if kpp_ms is not None:
            out["kmeanspp_ms"] = kpp_ms   # GPU k-means++ seeding of the same cloud (K centres), host prep included
            out["kmeanspp_cold_ms"] = kpp_cold_ms   # the process's first call (workspace allocation)
        if not args.no_cpu and world == 1:
            Xh, Ch = X.float().cpu().numpy(), C0.cpu().numpy()
            if args.config == 2:
                # the whole 20-iteration fit on the CPU and on the GPU, and their parity
                out["cpu_baseline"], ref = cpu_fit_baseline(Xh, Ch, args.steps)
                res = pcm_amd.lloyd_fit(X, C0, max_iter=args.steps, tol=0.0)
                torch.cuda.synchronize()
                out["parity_vs_cpu"] = {
                    "labels_bitwise": bool(np.array_equal(res.labels.cpu().numpy(), ref["labels"])),
                    "centres_bitwise": bool(np.array_equal(res.centers.cpu().numpy(), ref["centers"])),
                    "n_iter": [int(res.n_iter), int(ref["n_iter"])],
                    "inertia_equal": float(res.inertia) == ref["inertia"]}
            else:
                out["cpu_baseline"] = cpu_baseline(Xh, Ch)
            out["cpu_numpy"] = numpy_baseline(Xh, Ch)
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
