#!/bin/bash
# per-block phase timing of k_step for each variant: tools/step_sweep.sh "T1:512 T2:1024 ..."
for vb in $1; do v=${vb%%:*}; nb=${vb#*:}
  echo "== $v"; PCM_SO=$PWD/tools/variants/lib_$v.so timeout -k 10 200 python tools/step_timing.py $nb || exit 1
  PCM_SO=$PWD/tools/variants/lib_$v.so timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 3 | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", round(d["ms_per_step"]*1e3,1), "us/iter", {k: round(v*1e3,1) for k, v in d["breakdown_ms_per_iter"].items()})' || exit 1
done
