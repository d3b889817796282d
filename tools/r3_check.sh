#!/bin/bash
# Session check: GPU parity suite (parity + multirank + baseline sizes), k_step phase timing, bench lines.
set -o pipefail
T=gpurun_out/${1:-p3}; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest_gpu.txt 2>&1 || { tail -30 $T/pytest_gpu.txt; exit 1; }
tail -2 $T/pytest_gpu.txt
timeout -k 10 120 python tools/step_timing2.py $PWD/tools/variants/lib_dbgt.so 10 12500000 1024 3 > $T/st_s12.txt 2>&1 || { tail -5 $T/st_s12.txt; exit 1; }
grep -v amdgpu.ids $T/st_s12.txt
timeout -k 10 120 python tools/step_timing2.py $PWD/tools/variants/lib_dbgt.so 10 100000000 1024 3 > $T/st_c3.txt 2>&1 || { tail -5 $T/st_c3.txt; exit 1; }
grep -v amdgpu.ids $T/st_c3.txt
timeout -k 10 200 python bench.py --no-cpu > $T/bench.txt 2>&1 || { tail -20 $T/bench.txt; exit 1; }
tail -1 $T/bench.txt
timeout -k 10 200 python bench.py --no-cpu --split --n 12500000 > $T/split.txt 2>&1 || { tail -20 $T/split.txt; exit 1; }
tail -1 $T/split.txt
