"""Diagnose a linked-exchange mismatch: which words differ, and what they hold."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import pcm_amd
from pcm_amd import xchg

P, W = int(sys.argv[1]), int(sys.argv[2])
SYNC = len(sys.argv) > 3 and sys.argv[3] == "sync"
xs = xchg.linked(W, P)
g = torch.Generator(device="cuda").manual_seed(7)
hist = []
for rnd in range(4):
    bufs = [torch.randint(-2**40, 2**40, (W,), dtype=torch.int64, device="cuda", generator=g) for _ in range(P)]
    orig = [b.clone() for b in bufs]
    want = sum(orig)
    for r in range(P):
        xs[r].allreduce(bufs[r], 1)
    if SYNC:
        torch.cuda.synchronize()
    for r in range(P):
        xs[r].allreduce(bufs[r], 2)
    torch.cuda.synchronize()
    hist.append(orig)
    for r in range(P):
        bad = (bufs[r] != want).nonzero().flatten().cpu()
        if bad.numel():
            diff = (bufs[r] - want)[bad]
            # which peers' contributions are missing / stale?
            expl = []
            i0 = int(bad[0])
            for s in range(P):
                if s == r:
                    continue
                cur, prev = orig[s][i0], hist[-2][s][i0] if len(hist) > 1 else None
                expl.append((s, int(cur), None if prev is None else int(prev)))
            if len(hist) > 1:
                stale = orig[r][bad] + sum(hist[-2][s][bad] for s in range(P) if s != r)
                print("   bad words == own + previous round's peers:", bool(torch.equal(stale, bufs[r][bad])),
                      " bad blocks (512 words):", sorted(set((bad // 512).tolist())))
            print(f"rnd {rnd} rank {r}: {bad.numel()} bad words, first {int(bad[0])} last {int(bad[-1])}, "
                  f"diff at first {int(diff[0])}; peers (cur, prev) at first: {expl}")
    if SYNC:
        print("rnd", rnd, "status", [x.status() for x in xs])
