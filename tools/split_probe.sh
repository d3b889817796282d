#!/bin/bash
# One GPU: per-iteration time with/without per-kernel events, and through the
# multi-GPU call sequence (nccl group of 1), eager and graph-captured.
for n in 100000000 12500000; do
for a in "" "--no-events" "--split --no-events" "--split --graph"; do
  timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 3 --n $n $a > gpurun_out/sp.txt 2>&1 || { tail -20 gpurun_out/sp.txt; exit 1; }
  echo "[N=$n $a] $(tail -1 gpurun_out/sp.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,1), "us/iter", {k: round(v*1e3,1) for k, v in d["breakdown_ms_per_iter"].items()})')"
done; done
