#!/bin/bash
# per-iteration breakdown at shard sizes and the config-5 shape (one GPU)
set -o pipefail
mkdir -p gpurun_out/p
run() { local tag=$1; shift; timeout -k 10 150 python bench.py --no-cpu --fit-iters 0 "$@" > gpurun_out/p/$tag.json 2> gpurun_out/p/$tag.err || { tail -5 gpurun_out/p/$tag.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/p/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['ms_per_step']*1000,1), 'us/iter', d['breakdown_ms_per_iter'], d['candidates'], d['config']['cells'], d['config']['tiles'])"; }
run s12 --split --n 12500000
run s25 --split --n 25000000
run c5 --n 62500000 --k 4096 --d 4 --steps 10
