#!/bin/bash
# pruning-grid size sweep: tools/cell_sweep.sh N target1 target2 ...
mkdir -p gpurun_out/cells
n=$1; shift
for t in "$@"; do
  PCM_CELL_TARGET=$t timeout -k 10 120 python bench.py --no-cpu --fit-iters 0 --n $n > gpurun_out/cells/${n}_$t.txt 2>&1 || { tail -5 gpurun_out/cells/${n}_$t.txt; exit 1; }
  echo "$n $t $(tail -1 gpurun_out/cells/${n}_$t.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(r["avg_launch_ms"]*1e3,1), "us assign; step", round(d["ms_per_step"]*1e3,1), "us; update", round(d["breakdown_ms_per_iter"]["update"]*1e3,1), "cells", d["config"]["cells"], "cand", round(d["candidates"]["mean"],2), d["candidates"]["max"])')"
done
