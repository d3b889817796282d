#!/bin/bash
# points-per-tile sweep (PCM_TILE_CAP) at config 3 and on a 12.5M shard (multi-GPU call sequence)
mkdir -p gpurun_out/ts
for cap in 4096 2048 1536 1024; do
  for cfg in "c3|" "s12|--split --n 12500000"; do
    name=${cfg%%|*}; args=${cfg#*|}
    PCM_TILE_CAP=$cap timeout -k 10 120 python bench.py --no-cpu --fit-iters 0 $args > gpurun_out/ts/${name}_$cap.txt 2>&1 || { tail -5 gpurun_out/ts/${name}_$cap.txt; exit 1; }
    tail -1 gpurun_out/ts/${name}_$cap.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name cap=$cap', round(d['ms_per_step']*1e3,1), 'us/iter assign', round(d['breakdown_ms_per_iter']['assign']*1e3,1), 'tiles', d['config']['tiles'])"
  done
done
