#!/bin/bash
# pruning-grid size sweep at the 12.5M shard (split call sequence) and the config-5 shape
set -o pipefail
mkdir -p gpurun_out/w2
one() { local tag=$1; shift; env "$@" timeout -k 10 120 python bench.py --no-cpu --fit-iters 0 $ARGS > gpurun_out/w2/$tag.json 2> gpurun_out/w2/$tag.err || { tail -5 gpurun_out/w2/$tag.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/w2/$tag.json').read().strip().splitlines()[-1]); c=d['candidates']; print('$tag', round(d['ms_per_step']*1000,1), 'us/iter', {k: round(v*1000,1) for k, v in d['breakdown_ms_per_iter'].items()}, 'cells', d['config']['cells'], 'cand', round(c['mean'],2), c['max'])"; }
ARGS="--split --n 12500000"
for t in 4096 8000 13824 32768; do one s12_t$t PCM_CAND_BPC_RT=8 PCM_CELL_TARGET=$t; done
ARGS="--n 62500000 --k 4096 --d 4 --steps 10"
for t in 38416 65536; do one c5_t$t PCM_KSTEP_MAX=2048 PCM_CAND_BPC_RT=32 PCM_CELL_TARGET=$t; done
ARGS=""
for t in 32768 64000; do one c3_t$t PCM_CELL_TARGET=$t; done
