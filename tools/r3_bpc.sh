#!/bin/bash
# k_lloyd blocks-per-CU sweep at config 3 (one tile per block at large values)
set -o pipefail
T=gpurun_out/${1:-bpc}; mkdir -p $T
for b in 0 4 8 16 32 200; do
  if [ $b = 0 ]; then unset PCM_ASSIGN_BLOCKS_PER_CU; else export PCM_ASSIGN_BLOCKS_PER_CU=$b; fi
  timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 --no-graph > $T/b$b.txt 2>&1 || { tail -5 $T/b$b.txt; exit 1; }
  tail -1 $T/b$b.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bpc $b', round(d['ms_per_step']*1e3,1), {k: round(v*1e3,1) for k,v in d['breakdown_ms_per_iter'].items()})"
done
