#!/bin/bash
set -o pipefail
T=gpurun_out/${1:-mask}; mkdir -p $T
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_baseline_sizes.py -m gpu -x -q --timeout 200 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -30 $T/pytest.txt; exit 1; }
tail -1 $T/pytest.txt
run() { local tag=$1; shift; timeout -k 10 150 python bench.py --no-cpu --fit-iters 0 "$@" > $T/$tag.txt 2>&1 || { tail -5 $T/$tag.txt; exit 1; }
  tail -1 $T/$tag.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['ms_per_step']*1e3,1), {k: round(v*1e3,1) for k,v in d['breakdown_ms_per_iter'].items()}, d['roofline']['frac'])"; }
run c3
run s12 --split --n 12500000
run c5 --n 62500000 --k 4096 --d 4 --steps 10
timeout -k 10 120 python tools/lloyd_timing.py $PWD/tools/variants/lib_dbgt.so 10 12500000 1024 3 > $T/lt_s12.txt 2>&1 || { tail -5 $T/lt_s12.txt; exit 1; }
grep -v amdgpu.ids $T/lt_s12.txt | head -8
