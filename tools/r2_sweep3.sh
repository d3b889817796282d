#!/bin/bash
# resident assign blocks per CU at the 12.5M shard
set -o pipefail
mkdir -p gpurun_out/w3
one() { local tag=$1; shift; env "$@" timeout -k 10 120 python bench.py --no-cpu --fit-iters 0 $ARGS > gpurun_out/w3/$tag.json 2> gpurun_out/w3/$tag.err || { tail -5 gpurun_out/w3/$tag.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/w3/$tag.json').read().strip().splitlines()[-1]); c=d['candidates']; print('$tag', round(d['ms_per_step']*1000,1), 'us/iter', {k: round(v*1000,1) for k, v in d['breakdown_ms_per_iter'].items()}, 'cells', d['config']['cells'], 'cand', round(c['mean'],2), c['max'])"; }
ARGS="--split --n 12500000"
for b in 2 4 6 8 12; do one s12_pc$b PCM_ASSIGN_BLOCKS_PER_CU=$b; done
for b in 4 6; do one s12_pc${b}_t8000 PCM_ASSIGN_BLOCKS_PER_CU=$b PCM_CELL_TARGET=8000; done
