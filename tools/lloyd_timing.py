"""Calibration (debug build -DPCM_DBG_TIMING): per-block phase times of the
k_lloyd1 launch of the last of `iters` iterations.
usage: python tools/lloyd_timing.py SO_PATH [iters] [N K D [f16] [slab P]]  (default config 3)
  slab P: time rank 0's spatial slab of a P-way split (the layout bench.py --slab-of P
  and the multi-GPU run use) instead of a whole-cloud engine"""
import ctypes, os, sys
import numpy as np
os.environ["PCM_SO"] = sys.argv[1]
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pcm_amd import lloyd, _lib
from pcm_amd.engine import Engine, shard_hist, shard_partition, synth_rows, synth_uniform
from pcm_amd.fixed import fixed_q
rest = sys.argv[3:]
N, K, D = (int(v) for v in rest[:3]) if len(rest) >= 3 else (100_000_000, 1024, 3)
pdt = torch.float16 if "f16" in rest else torch.float32
P = int(rest[rest.index("slab") + 1]) if "slab" in rest else 1
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
X = synth_uniform(N, D, seed=0, start=0).to(pdt)
C0 = synth_rows(np.sort(np.random.default_rng(1).choice(N, K, replace=False)), D, seed=0).to(pdt).float()
eng = Engine(D, K, pdt, max_iter=50)
if P > 1:   # rank 0's slab, built as bench.slab_proxy does
    lo, hi, maxabs = Engine(D, K, pdt, max_iter=1).bbox(X)
    q = fixed_q(maxabs)
    axis = int(np.argmax(hi - lo))
    inv = lloyd.SLAB_BINS / (hi[axis] - lo[axis])
    owner = lloyd.slab_owner(shard_hist(X, axis, lo[axis], inv, lloyd.SLAB_BINS).cpu().numpy(), P)
    Xp, rows, cnt = shard_partition(X, axis, lo[axis], inv, lloyd.SLAB_BINS, owner, P, 0)
    Xr, rr = Xp[:int(cnt[0])].contiguous(), rows[:int(cnt[0])].contiguous()
    del X, Xp
    eng.bbox(Xr)
    eng.set_shard(rr, N)
    eng.build(Xr, q, 0)
else:
    lloyd.prepare(eng, X, None)
eng.begin(C0, 0.0, 50)
eng.iterate(iters); torch.cuda.synchronize()
lib = _lib.load()
lib.pcm_debug_timing_lloyd.argtypes = [ctypes.c_void_p, ctypes.c_int]
nb = 65536
buf = np.zeros((nb, 8), np.uint64)
assert lib.pcm_debug_timing_lloyd(buf.ctypes.data_as(ctypes.c_void_p), nb) == 0
t = buf.astype(np.int64)
t = t[t[:, 0] > 0]
# columns: 0 record in (after the block's first memory latency), 1 first round, 2 rounds done,
# 3 end, 5 HW_ID, 6 XCC_ID, 7 list length | tile points << 16 (a stamp before the first loads
# trips hipcc: "illegal VGPR to SGPR copy")
t0 = t[:, 0].min()
us = lambda v: np.asarray(v) / 100.0   # s_memrealtime: 100 MHz
info = eng.layout_info()
print(f"N={N} K={K} D={D} {pdt} slab {P} (rank 0: {int(eng.n)} points, cells {info['ncells']}, tiles "
      f"{info['ntiles']}, kernel {eng.assign_kernel()}, lists {eng.candidate_stats()}) blocks {len(t)} "
      f"kernel span {us(t[:, 3].max() - t0):.1f} us")
for name, a, b in (("start (rel. first)", None, 0), ("setup (record->first round)", 0, 1), ("rounds", 1, 2),
                   ("fold+exit", 2, 3), ("block total", 0, 3), ("end (rel. first start)", None, 3)):
    v = t[:, b] - (t0 if a is None else t[:, a])
    print("%-28s p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f us" % ((name,) + tuple(us(np.percentile(v, q)) for q in (10, 50, 90, 100))))
# concurrency: blocks resident over time (1 us bins)
span = int(us(t[:, 3].max() - t0)) + 1
occ = np.zeros(span + 1)
for s_, e_ in zip(us(t[:, 0] - t0).astype(int), us(t[:, 3] - t0).astype(int)):
    occ[s_:e_ + 1] += 1
print("resident blocks per us bin:", " ".join(str(int(x)) for x in occ[::max(1, span // 40)]))

# what the slow blocks have in common: block time by XCC, shader engine, list length, tile size, start time
tot = us(t[:, 3] - t[:, 0])
rnd = us(t[:, 2] - t[:, 1])
xcc = t[:, 6] & 0xF
se = (t[:, 5] >> 13) & 0x7
mm = t[:, 7] & 0xFFFF
ln = (t[:, 7] >> 16) & 0xFFFF
st = us(t[:, 0] - t0)
def by(name, key, vals):
    out = []
    for v in vals:
        m = key == v
        if m.sum():
            out.append(f"{v}:{tot[m].mean():.1f}/{rnd[m].mean():.1f}({m.sum()})")
    print(f"block total/rounds mean by {name}: " + " ".join(out))
by("xcc", xcc, range(8))
by("se", se, range(8))
by("list len", np.minimum(mm, 12), range(13))
q = np.quantile(ln, [0.0, 0.25, 0.5, 0.75, 1.0])
by("tile pts quartile", np.searchsorted(q[1:-1], ln), range(4))
by("start us//4", np.minimum(st // 4, 12).astype(int), range(13))
print("corr(total, list len) %.2f  corr(total, tile pts) %.2f  corr(rounds, start) %.2f" % (
    np.corrcoef(tot, mm)[0, 1], np.corrcoef(tot, ln)[0, 1], np.corrcoef(rnd, st)[0, 1]))
