#!/bin/bash
# assign block size x grid size sweep: libraries tools/variants/lib_tpb{128,256}.so
mkdir -p gpurun_out/tpb
for spec in "100000000 0" "100000000 65536" "12500000 0" "12500000 8000" "12500000 16000" "62500000 0"; do
  set -- $spec; n=$1; t=$2
  for v in tpb256 tpb128; do
    env=""; [ "$t" != "0" ] && export PCM_CELL_TARGET=$t || unset PCM_CELL_TARGET
    extra=""; [ "$n" = "62500000" ] && extra="--k 4096 --d 4"
    PCM_SO=$PWD/tools/variants/lib_$v.so timeout -k 10 120 python bench.py --no-cpu --fit-iters 0 --n $n $extra > gpurun_out/tpb/${v}_${n}_$t.txt 2>&1 || { tail -3 gpurun_out/tpb/${v}_${n}_$t.txt; exit 1; }
    echo "$n cells~$t $v $(tail -1 gpurun_out/tpb/${v}_${n}_$t.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(r["avg_launch_ms"]*1e3,1), "us assign; step", round(d["ms_per_step"]*1e3,1), "us; cells", d["config"]["cells"], "cand", round(d["candidates"]["mean"],2))')"
  done
done
