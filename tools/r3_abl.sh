#!/bin/bash
# ablations of k_lloyd at config 3 (assign time per launch, HIP events) + stream probe
set -o pipefail
T=gpurun_out/${1:-abl}; mkdir -p $T
timeout -k 10 60 ./tools/stream_probe > $T/stream.txt 2>&1 || exit 1
cat $T/stream.txt
for v in base noscan noacc both noflush; do
  if [ $v = base ]; then so=""; else so=$PWD/tools/variants/lib_$v.so; fi
  PCM_SO=$so timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 --no-graph > $T/$v.txt 2>&1 || { tail -5 $T/$v.txt; exit 1; }
  tail -1 $T/$v.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step']*1e3,1), {k: round(v*1e3,1) for k,v in d['breakdown_ms_per_iter'].items()})"
done
