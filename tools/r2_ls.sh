#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/p
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/p/ls_tests.log 2>&1; rc=$?; tail -3 gpurun_out/p/ls_tests.log; [ $rc = 0 ] || exit $rc
for n in 100000000 12500000; do
  timeout -k 10 120 python bench.py --no-cpu --fit-iters 0 --n $n > gpurun_out/p/ls_$n.json 2> gpurun_out/p/ls_$n.err || { tail -5 gpurun_out/p/ls_$n.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/p/ls_$n.json').read().strip().splitlines()[-1]); print($n, round(d['ms_per_step']*1000,1), 'us/iter', d['breakdown_ms_per_iter'], d['roofline']['frac'])"
done
