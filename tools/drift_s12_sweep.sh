#!/bin/bash
# candidate-list reuse policy on a 12.5M shard and at config 3: kappa (budget cap, cell widths) x alpha
mkdir -p gpurun_out/ds
for cfg in "0.05 2" "0.2 2" "0.5 2" "0.5 1.5" "1.0 2"; do
  set -- $cfg
  for w in "s12|--split --n 12500000" "c3|"; do
    name=${w%%|*}; args=${w#*|}
    PCM_DRIFT_KAPPA=$1 PCM_DRIFT_ALPHA=$2 timeout -k 10 120 python bench.py --no-cpu --fit-iters 0 $args > gpurun_out/ds/${name}_$1_$2.txt 2>&1 || { tail -5 gpurun_out/ds/${name}_$1_$2.txt; exit 1; }
    tail -1 gpurun_out/ds/${name}_$1_$2.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name kappa=$1 alpha=$2', round(d['ms_per_step']*1e3,1), 'us/iter assign', round(d['breakdown_ms_per_iter']['assign']*1e3,1), 'cand', round(d['candidates']['mean'],2), 'rebuilds', d['candidates']['list_rebuilds'], '/', d['candidates']['iterations'])"
  done
done
