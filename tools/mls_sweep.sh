#!/bin/bash
# (the PCM_MASK_LS switch was removed after this sweep: 12 slots measured 42.6 -> 65.7 us)
# coarse-grid (12.5M shard) masked k_lloyd1: 16 vs 12 lane slots (PCM_MASK_LS)
mkdir -p gpurun_out/ml
for r in 1 2; do for v in 16 12; do
  PCM_MASK_LS=$v timeout -k 10 120 python bench.py --no-cpu --fit-iters 0 --split --n 12500000 > gpurun_out/ml/s12_$v.txt 2>&1 || { tail -5 gpurun_out/ml/s12_$v.txt; exit 1; }
  tail -1 gpurun_out/ml/s12_$v.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('mask_ls=$v s12', round(d['ms_per_step']*1e3,1), 'us/iter assign', round(d['breakdown_ms_per_iter']['assign']*1e3,1))"
done; done
