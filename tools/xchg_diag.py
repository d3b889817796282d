"""Replay test_linked_allreduce_exact's sequence with diagnostics on a mismatch."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import pcm_amd  # noqa: F401
from pcm_amd import xchg

def case(P, words, diag):
    xs = xchg.linked(words, P)
    g = torch.Generator(device="cuda").manual_seed(P * 1000 + words)
    prev = None
    for rnd in range(5):
        bufs = [torch.randint(-2**62, 2**62, (words,), dtype=torch.int64, device="cuda", generator=g) for _ in range(P)]
        orig = [b.clone() for b in bufs]
        want = sum(b.clone() for b in bufs)
        for r in range(P):
            xs[r].allreduce(bufs[r], 1)
        for r in range(P):
            xs[r].allreduce(bufs[r], 2)
        torch.cuda.synchronize()
        for r in range(P):
            if not torch.equal(bufs[r], want):
                bad = (bufs[r] != want).nonzero().flatten()
                print(f"P={P} W={words} rnd {rnd} rank {r}: {bad.numel()} bad, blocks {sorted(set((bad // 512).tolist()))[:20]}")
                if diag and prev is not None:
                    got = bufs[r][bad]
                    stale = orig[r][bad] + sum(prev[s][bad] for s in range(P) if s != r)
                    print("  == own + previous round's peers:", bool(torch.equal(stale, got)))
                    for s in range(P):
                        if s == r:
                            continue
                        miss = want[bad] - orig[s][bad] + prev[s][bad]
                        if torch.equal(miss, got):
                            print("  == sender", s, "stale")
                    print("  xs status", [x.status() for x in xs])
                return False
        prev = orig
    print(f"P={P} W={words} ok", [x.status()["epoch"] for x in xs])
    return True

for P, W in [(2, 4097), (3, 1), (3, 4096), (8, 4097), (8, 20481), (16, 257)]:
    case(P, W, True)
print("alone:")
case(8, 20481, True)
