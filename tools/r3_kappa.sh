#!/bin/bash
# drift-budget cap sweep (candidate-list reuse): config 3 and a 12.5M shard
set -o pipefail
T=gpurun_out/${1:-kap}; mkdir -p $T
run() { local tag=$1; shift; timeout -k 10 150 python bench.py --no-cpu --fit-iters 0 "$@" > $T/$tag.txt 2>&1 || { tail -5 $T/$tag.txt; exit 1; }
  tail -1 $T/$tag.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['ms_per_step']*1e3,1), {k: round(v*1e3,1) for k,v in d['breakdown_ms_per_iter'].items()}, round(d['candidates']['mean'],2), d['candidates']['list_rebuilds'], d['candidates']['iterations'])"; }
for k in 0.05 0.1 0.2 0.4; do
  PCM_DRIFT_KAPPA=$k run c3_k$k
  PCM_DRIFT_KAPPA=$k run s12_k$k --split --n 12500000
done
