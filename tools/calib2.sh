#!/bin/bash
# assign-kernel ablation builds at two cloud sizes: tools/calib2.sh v1 v2 ...
mkdir -p gpurun_out/calib
for n in 100000000 12500000; do for v in "$@"; do
  PCM_SO=$PWD/tools/variants/lib_$v.so timeout -k 10 120 python bench.py --no-cpu --fit-iters 0 --n $n > gpurun_out/calib/${v}_$n.txt 2>&1 || { tail -5 gpurun_out/calib/${v}_$n.txt; exit 1; }
  echo "$n $v $(tail -1 gpurun_out/calib/${v}_$n.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(r["avg_launch_ms"]*1e3,1), "us", round(r["achieved"]), "GB/s step_ms", round(d["ms_per_step"],3))')"
done; done
