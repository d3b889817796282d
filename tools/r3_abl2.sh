#!/bin/bash
# k_lloyd1 ablations at config 3 and a 12.5M shard (assign time per launch, HIP events)
set -o pipefail
T=gpurun_out/${1:-abl}; mkdir -p $T
for v in base noscan noacc; do
  if [ $v = base ]; then so=""; else so=$PWD/tools/variants/lib_$v.so; fi
  for cfg in "c3 100000000" "s12 12500000"; do set -- $cfg
  PCM_SO=$so timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 --no-graph --n $2 > $T/${v}_$1.txt 2>&1 || { tail -5 $T/${v}_$1.txt; exit 1; }
  tail -1 $T/${v}_$1.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $1', round(d['ms_per_step']*1e3,1), {k: round(v*1e3,1) for k,v in d['breakdown_ms_per_iter'].items()}, d['candidates']['mean'])"
  done
done
