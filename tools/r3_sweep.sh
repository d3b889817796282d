#!/bin/bash
# k_lloyd launch geometry sweep: default vs one tile per block (bpc 200), TPB 128 vs 256; c3, 12.5M split, c5 shape
set -o pipefail
T=gpurun_out/${1:-sw}; mkdir -p $T
run() { local tag=$1; shift; timeout -k 10 150 python bench.py --no-cpu --fit-iters 0 --no-graph "$@" > $T/$tag.txt 2>&1 || { tail -5 $T/$tag.txt; exit 1; }
  tail -1 $T/$tag.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['ms_per_step']*1e3,1), {k: round(v*1e3,1) for k,v in d['breakdown_ms_per_iter'].items()}, round(d['candidates']['mean'],2))"; }
for so in "" $PWD/tools/variants/lib_tpb256.so; do
  for b in 0 200; do
    if [ $b = 0 ]; then unset PCM_ASSIGN_BLOCKS_PER_CU; else export PCM_ASSIGN_BLOCKS_PER_CU=$b; fi
    tag=$(basename ${so:-base} .so)_b$b
    PCM_SO=$so run c3_$tag
    PCM_SO=$so run s12_$tag --n 12500000
    PCM_SO=$so run c5_$tag --n 62500000 --k 4096 --d 4 --steps 10
  done
done
