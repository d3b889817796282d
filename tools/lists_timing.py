"""Calibration (debug build -DPCM_DBG_TIMING): per-block phase times of the
last k_lists launch (cand_body's DBG_T marks) after `iters` iterations.
usage: python tools/lists_timing.py SO_PATH iters N K D [f16] [slab P]"""
import ctypes, os, sys
import numpy as np
os.environ["PCM_SO"] = sys.argv[1]
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pcm_amd import lloyd, _lib
from pcm_amd.engine import Engine, shard_hist, shard_partition, synth_rows, synth_uniform
from pcm_amd.fixed import fixed_q
iters = int(sys.argv[2])
rest = sys.argv[3:]
N, K, D = (int(v) for v in rest[:3])
pdt = torch.float16 if "f16" in rest else torch.float32
P = int(rest[rest.index("slab") + 1]) if "slab" in rest else 1
FUSED = "fused" in sys.argv[3:]
os.environ.setdefault("PCM_FUSED_UPD", "1" if FUSED else "0")   # D <= 3: k_lists, or (fused) k_updlists
X = synth_uniform(N, D, seed=0, start=0).to(pdt)
C0 = synth_rows(np.sort(np.random.default_rng(1).choice(N, K, replace=False)), D, seed=0).to(pdt).float()
eng = Engine(D, K, pdt, max_iter=50) if P == 1 else None
if P > 1:   # the P slab engines of bench.py --slab-of P; the stamps are those of the last engine's launch
    lo, hi, maxabs = Engine(D, K, pdt, max_iter=1).bbox(X)
    q = fixed_q(maxabs)
    axis = int(np.argmax(hi - lo))
    inv = lloyd.SLAB_BINS / (hi[axis] - lo[axis])
    owner = lloyd.slab_owner(shard_hist(X, axis, lo[axis], inv, lloyd.SLAB_BINS).cpu().numpy(), P)
    Xp, rows, cnt = shard_partition(X, axis, lo[axis], inv, lloyd.SLAB_BINS, owner, P, 0)
    del X
    engines, off = [], 0
    for r in range(P):
        e = Engine(D, K, pdt, max_iter=50)
        Xr, rr = Xp[off:off + int(cnt[r])], rows[off:off + int(cnt[r])]
        off += int(cnt[r])
        e.bbox(Xr)
        e.set_shard(rr, N)
        e.build(Xr, q, 0)
        e.begin(C0, 0.0, 50)
        engines.append(e)
    del Xp
    for _ in range(iters):
        for e in engines:
            e.iter_local()
        total = engines[0].stats.clone()
        for e in engines[1:]:
            total += e.stats
        for e in engines:
            e.stats.copy_(total)
        for e in engines:
            e.iter_global()
    torch.cuda.synchronize()
    eng = engines[-1]
else:
    lloyd.prepare(eng, X, None)
    eng.begin(C0, 0.0, 50)
    eng.iterate(iters); torch.cuda.synchronize()
st = eng.status()
lib = _lib.load()
lib.pcm_debug_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
nb = 8192
buf = np.zeros((nb, 16), np.uint64)
assert lib.pcm_debug_timing(buf.ctypes.data_as(ctypes.c_void_p), nb) == 0
t = buf.astype(np.int64)
t = t[t[:, 0] > 0]
t0 = t[:, 0].min()
us = lambda v: np.asarray(v) / 100.0   # s_memrealtime: 100 MHz
print(f"N={N} K={K} D={D} slab {P}: iters {st['iter']} rebuilds {st['list_rebuilds']} blocks {len(t)} "
      f"layout {eng.layout_info()} lists {eng.candidate_stats()}")
t0 = t[:, 13].min() if FUSED else t0
print("block start rel. first us: p50 %.1f p90 %.1f max %.1f" % tuple(us(np.percentile(t[:, 13 if FUSED else 0] - t0, q)) for q in (50, 90, 100)))
# fused marks since round 5: 15 centres + decisions done, 14 lists start, 2 lists done, 3 arrival
# returned (after the lists), 6 the publisher's end (one block per launch: 6 > 3 in its row)
for k0, k1, name in ((13, 0, "fused: control + rows (one latency)"), (0, 15, "fused: centres + decisions"),
                     (15, 14, "fused: -> lists"), (14, 4, "fused: -> list reference"),
                     (2, 3, "fused: arrival (after lists)"), (3, 6, "fused: publisher"),
                     (0, 4, "list source + reference"), (4, 5, "prune bits"), (5, 1, "compaction"), (1, 10, "children boxes"),
                     (10, 11, "pair A (refs)"), (11, 12, "pair B (prune)"), (12, 2, "pair C (write)"), (0, 2, "block total")):
    ok = (t[:, k0] > 0) & (t[:, k1] > t[:, k0] if (k0, k1) == (3, 6) else t[:, k1] > 0)
    if ok.any():
        dd = t[ok, k1] - t[ok, k0]
        print("%-24s us: p50 %6.2f p90 %6.2f max %6.2f (%d blocks)" % (name, us(np.median(dd)), us(np.percentile(dd, 90)), us(dd.max()), ok.sum()))
print("last block end rel. first start: %.1f us" % us(max(t[:, 2].max(), t[:, 3].max()) - t0))
print("list length (mark 8) p10/p50/p90/max:", [int(np.percentile(t[:, 8], q)) for q in (10, 50, 90, 100)])
