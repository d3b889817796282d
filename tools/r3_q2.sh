#!/bin/bash
set -o pipefail
T=gpurun_out/${1:-q}; mkdir -p $T
bash tools/r3_quick.sh $1 || exit 1
timeout -k 10 120 python tools/lloyd_timing.py $PWD/tools/variants/lib_dbgt.so 10 100000000 1024 3 > $T/lt_c3.txt 2>&1 || { tail -5 $T/lt_c3.txt; exit 1; }
grep -v amdgpu.ids $T/lt_c3.txt
timeout -k 10 120 python tools/lloyd_timing.py $PWD/tools/variants/lib_dbgt.so 10 12500000 1024 3 > $T/lt_s12.txt 2>&1 || { tail -5 $T/lt_s12.txt; exit 1; }
grep -v amdgpu.ids $T/lt_s12.txt
timeout -k 10 150 python bench.py --no-cpu --fit-iters 0 --n 62500000 --k 4096 --d 4 --steps 10 > $T/c5.txt 2>&1 || { tail -5 $T/c5.txt; exit 1; }
tail -1 $T/c5.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', d['ms_per_step'], d['breakdown_ms_per_iter'])"
