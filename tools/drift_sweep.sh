#!/bin/bash
# drift-budget sweep on the headline workload
mkdir -p gpurun_out/sw
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sw/pytest.txt 2>&1; tail -3 gpurun_out/sw/pytest.txt
for cfg in "0 0.5" "2 0.5" "3 0.5" "5 0.5" "3 0.25" "3 1.0" "8 1.0"; do
  set -- $cfg
  PCM_DRIFT_ALPHA=$1 PCM_DRIFT_KAPPA=$2 timeout -k 10 120 python bench.py --no-cpu --fit-iters 0 > gpurun_out/sw/b_$1_$2.txt 2>&1 || { echo fail $cfg; tail -5 gpurun_out/sw/b_$1_$2.txt; exit 1; }
  python -c "
import json,sys; d=json.loads(open('gpurun_out/sw/b_$1_$2.txt').read().strip().splitlines()[-1]); print('$1 $2', round(d['ms_per_step'],4), d['breakdown_ms_per_iter'], d['candidates'])"
done
