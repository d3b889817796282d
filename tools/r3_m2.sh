#!/bin/bash
# tiles per block 1 vs 2: parity subset, 12.5M shard (split), config 3, config-5 shape; block timing at 12.5M
set -o pipefail
T=gpurun_out/${1:-m2}; mkdir -p $T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -30 $T/pytest.txt; exit 1; }
tail -1 $T/pytest.txt
run() { local tag=$1; shift; timeout -k 10 150 python bench.py --no-cpu --fit-iters 0 "$@" > $T/$tag.txt 2>&1 || { tail -5 $T/$tag.txt; exit 1; }
  tail -1 $T/$tag.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['ms_per_step']*1e3,1), {k: round(v*1e3,1) for k,v in d['breakdown_ms_per_iter'].items()})"; }
for m in 1 2; do
  export PCM_TILES_PER_BLOCK=$m
  run s12_m$m --split --n 12500000
  run c3_m$m
  run c5_m$m --n 62500000 --k 4096 --d 4 --steps 10
  timeout -k 10 120 python tools/lloyd_timing.py $PWD/tools/variants/lib_dbgt.so 10 12500000 1024 3 > $T/lt_s12_m$m.txt 2>&1 || { tail -5 $T/lt_s12_m$m.txt; exit 1; }
  grep -v amdgpu.ids $T/lt_s12_m$m.txt
done
