#!/bin/bash
# multi-GPU call sequence on one GPU (nccl group of 1): per-iteration cost at shard sizes
mkdir -p gpurun_out/s
for n in 12500000 100000000; do for g in "--no-graph" ""; do
  timeout -k 10 120 python bench.py --no-cpu --fit-iters 0 --split $g --n $n > gpurun_out/s/b_${n}$g.txt 2>&1 || { tail -5 gpurun_out/s/b_${n}$g.txt; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/s/b_${n}$g.txt').read().strip().splitlines()[-1]); print('n=$n $g', round(d['ms_per_step']*1000,1), 'us/iter', d['breakdown_ms_per_iter'])"
done; done
