#!/bin/bash
# k_lloyd1 occupancy variants (amdgpu_waves_per_eu minimum): main build vs tools/variants/lib_$1.so
mkdir -p gpurun_out/wp
for so in main "$@"; do
  for cfg in "c3|" "s12|--split --n 12500000" "c5|--n 62500000 --k 4096 --d 4"; do
    name=${cfg%%|*}; args=${cfg#*|}
    if [ "$so" = main ]; then env=""; else env="PCM_SO=tools/variants/lib_$so.so"; fi
    env $env timeout -k 10 120 python bench.py --no-cpu --fit-iters 0 $args > gpurun_out/wp/${name}_$so.txt 2>&1 || { tail -5 gpurun_out/wp/${name}_$so.txt; exit 1; }
    tail -1 gpurun_out/wp/${name}_$so.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$so $name', round(d['ms_per_step']*1e3,1), 'us/iter assign', round(d['breakdown_ms_per_iter']['assign']*1e3,1))"
  done
done
