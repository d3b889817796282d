#!/bin/bash
# config-3 and config-5-shape bench lines + the GPU parity suite (one GPU)
set -o pipefail
mkdir -p gpurun_out/p
run() { local tag=$1; shift; timeout -k 10 150 python bench.py --no-cpu --fit-iters 0 "$@" > gpurun_out/p/$tag.json 2> gpurun_out/p/$tag.err || { tail -5 gpurun_out/p/$tag.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/p/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['ms_per_step']*1000,1), 'us/iter', d['breakdown_ms_per_iter'], d['candidates'], d['roofline']['frac'])"; }
run c5 --n 62500000 --k 4096 --d 4 --steps 10
run c3
if [ "$1" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py > gpurun_out/p/tests.log 2>&1; rc=$?; tail -3 gpurun_out/p/tests.log; exit $rc
fi
