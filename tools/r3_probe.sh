#!/bin/bash
# Session probe: GPU tests, k_step phase timing (12.5M shard, config 3), bench line.
set -o pipefail
T=gpurun_out/p3; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 120 python tools/step_timing2.py $PWD/tools/variants/lib_dbgt.so 10 12500000 1024 3 > $T/st_s12.txt 2>&1 || { tail -5 $T/st_s12.txt; exit 1; }
grep -v amdgpu.ids $T/st_s12.txt
timeout -k 10 120 python tools/step_timing2.py $PWD/tools/variants/lib_dbgt.so 10 100000000 1024 3 > $T/st_c3.txt 2>&1 || { tail -5 $T/st_c3.txt; exit 1; }
grep -v amdgpu.ids $T/st_c3.txt
timeout -k 10 200 python bench.py --no-cpu > $T/bench.txt 2>&1 || { tail -20 $T/bench.txt; exit 1; }
tail -1 $T/bench.txt
timeout -k 10 200 python bench.py --no-cpu --split --n 12500000 > $T/split.txt 2>&1 || { tail -20 $T/split.txt; exit 1; }
tail -1 $T/split.txt
