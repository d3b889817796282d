#!/bin/bash
# k_lloyd per-block timing (12.5M shard, config 3) + k_step phases
set -o pipefail
T=gpurun_out/${1:-lt}; mkdir -p $T
L=$PWD/tools/variants/lib_dbgt.so
for cfg in "s12 12500000 1024 3" "c3 100000000 1024 3"; do
  set -- $cfg
  timeout -k 10 120 python tools/lloyd_timing.py $L 10 $2 $3 $4 > $T/lt_$1.txt 2>&1 || { tail -5 $T/lt_$1.txt; exit 1; }
  grep -v amdgpu.ids $T/lt_$1.txt
  timeout -k 10 120 python tools/step_timing2.py $L 10 $2 $3 $4 > $T/st_$1.txt 2>&1 || { tail -5 $T/st_$1.txt; exit 1; }
  grep -v amdgpu.ids $T/st_$1.txt
done
