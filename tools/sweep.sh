#!/bin/bash
# usage: tools/sweep.sh VAR "v1 v2 ..." [bench args]   -> one line per value: value, assign us, GB/s
VAR=$1; VALS=$2; shift 2
for v in $VALS; do
  out=$(env $VAR=$v timeout -k 10 200 python bench.py --no-cpu "$@" 2>/dev/null | grep '^{')
  echo "$VAR=$v $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(r["avg_launch_ms"]*1e3,1), "us", round(r["achieved"]), "GB/s", "step_ms", round(d["ms_per_step"],3))')"
done
