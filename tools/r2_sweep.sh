#!/bin/bash
# k_step geometry sweep: blocks per coarse cell (PCM_CAND_BPC_RT) x fused-step limit (PCM_KSTEP_MAX)
set -o pipefail
mkdir -p gpurun_out/w
one() { local tag=$1; shift; env "$@" timeout -k 10 120 python bench.py --no-cpu --fit-iters 0 $ARGS > gpurun_out/w/$tag.json 2> gpurun_out/w/$tag.err || { tail -5 gpurun_out/w/$tag.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/w/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['ms_per_step']*1000,1), 'us/iter', {k: round(v*1000,1) for k, v in d['breakdown_ms_per_iter'].items()})"; }
ARGS="--split --n 12500000"
for b in 4 8 16 32; do one s12_b$b PCM_CAND_BPC_RT=$b; done
ARGS="--n 62500000 --k 4096 --d 4 --steps 10"
for km in 2048 4096; do for b in 8 16 32; do one c5_k${km}_b$b PCM_KSTEP_MAX=$km PCM_CAND_BPC_RT=$b; done; done
