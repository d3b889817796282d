"""Cold-start probe: the first lloyd.prepare (layout) of a process vs later ones.

Prints, per trial, the wall time of lloyd.prepare on a fresh engine and on the
same engine again, host-side intervals of the first layout's steps, and (with
PCM_RESERVE=1) the effect of Engine.reserve(N) before each layout.  Run it under rocprofv3
--kernel-trace to see the gaps between the first layout's kernels.

usage: python tools/cold_start_probe.py [N] [K] [D]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    d = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    t0 = time.perf_counter()
    import torch
    torch.cuda.init()
    t1 = time.perf_counter()
    from pcm_amd import lloyd
    from pcm_amd.engine import Engine, synth_uniform
    t2 = time.perf_counter()
    X = synth_uniform(n, d, seed=0)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    print(f"torch init {1e3 * (t1 - t0):.1f} ms, import pcm_amd {1e3 * (t2 - t1):.1f} ms, "
          f"first synth {1e3 * (t3 - t2):.1f} ms", flush=True)
    for trial in range(3):
        t = time.perf_counter()
        eng = Engine(d, k, torch.float32, max_iter=8)
        torch.cuda.synchronize()
        if os.environ.get("PCM_RESERVE") == "1":
            tr = time.perf_counter()
            eng.reserve(n)
            torch.cuda.synchronize()
            print(f"trial {trial}: reserve {1e3 * (time.perf_counter() - tr):.2f} ms", flush=True)
        tc = time.perf_counter()
        m0 = time.monotonic_ns()
        lloyd.prepare(eng, X, lloyd.LOCAL)
        torch.cuda.synchronize()
        tl = time.perf_counter()
        m1 = time.monotonic_ns()
        lloyd.prepare(eng, X, lloyd.LOCAL)
        torch.cuda.synchronize()
        tl2 = time.perf_counter()
        print(f"trial {trial}: engine create {1e3 * (tc - t):.2f} ms, layout (fresh engine) {1e3 * (tl - tc):.2f} ms, "
              f"layout again {1e3 * (tl2 - tl):.2f} ms; first layout CLOCK_MONOTONIC ns [{m0}, {m1}]", flush=True)
        del eng


if __name__ == "__main__":
    main()
