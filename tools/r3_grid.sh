#!/bin/bash
# grid / slot sweep with k_lloyd1 + new k_step: 12.5M shard (split sequence) and config 3
set -o pipefail
T=gpurun_out/${1:-grid}; mkdir -p $T
run() { local tag=$1; shift; timeout -k 10 150 python bench.py --no-cpu --fit-iters 0 "$@" > $T/$tag.txt 2>&1 || { tail -5 $T/$tag.txt; exit 1; }
  tail -1 $T/$tag.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['ms_per_step']*1e3,1), {k: round(v*1e3,1) for k,v in d['breakdown_ms_per_iter'].items()}, d['config']['cells'], round(d['candidates']['mean'],2))"; }
for tgt in 4096 5832 8000 13824; do
  for ls in 16 8; do
    PCM_CELL_TARGET=$tgt PCM_LSLOT_RT=$ls run s12_t${tgt}_ls$ls --split --n 12500000
  done
done
for tgt in 27000 32768 46656; do
  PCM_CELL_TARGET=$tgt run c3_t$tgt
done
