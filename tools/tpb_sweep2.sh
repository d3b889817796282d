#!/bin/bash
# assign-kernel geometry variants (tools/variants/lib_*.so) at three shapes
mkdir -p gpurun_out/tpb2
for spec in "100000000" "12500000" "62500000"; do
  n=$spec; extra=""; [ "$n" = "62500000" ] && extra="--k 4096 --d 4"
  for v in "$@"; do
    PCM_SO=$PWD/tools/variants/lib_$v.so timeout -k 10 120 python bench.py --no-cpu --fit-iters 0 --n $n $extra > gpurun_out/tpb2/${v}_${n}.txt 2>&1 || { tail -3 gpurun_out/tpb2/${v}_${n}.txt; exit 1; }
    echo "$n $v $(tail -1 gpurun_out/tpb2/${v}_${n}.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(r["avg_launch_ms"]*1e3,1), "us assign; step", round(d["ms_per_step"]*1e3,1), "us; cand", round(d["candidates"]["mean"],2))')"
  done
done
