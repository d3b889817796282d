#!/bin/bash
set -o pipefail
T=gpurun_out/${1:-st}; mkdir -p $T
L=$PWD/tools/variants/lib_dbgt.so
for cfg in "s12 12500000 1024 3" "c3 100000000 1024 3"; do
  set -- $cfg
  timeout -k 10 120 python tools/step_timing2.py $L 10 $2 $3 $4 > $T/st_$1.txt 2>&1 || { tail -5 $T/st_$1.txt; exit 1; }
  grep -v amdgpu.ids $T/st_$1.txt
done
