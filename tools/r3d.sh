#!/bin/bash
# round 3: rocprof kernel stats of (a) the counting-sort layout bench, (b) the 8-way slab proxy, (c) the 12.5M row shard
T=gpurun_out/r3d; mkdir -p $T
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
prof() {  # name, bench args
  local N=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/$N -o run -- python3 bench.py "$@" > $T/$N.txt 2>&1 || { tail -20 $T/$N.txt; return 1; }
  local f=$(find $T/$N -name "*kernel_stats.csv" | head -1); cp "$f" $T/${N}_kernel_stats.csv
  python3 - "$T/${N}_kernel_stats.csv" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    print(f'{r["Name"][:60]:60s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:9.2f} min_us={float(r["MinNs"])/1e3:9.2f} pct={r["Percentage"]}')
PY
}
echo "== counting-sort layout (bench, fit)"; prof count --no-cpu --steps 20 --warmup 3 || exit 1
echo "== slab proxy 8"; prof proxy8 --slab-of 8 --steps 20 --warmup 3 || exit 1
echo "== row shard 12.5M split"; prof rows --split --no-cpu --fit-iters 0 --n 12500000 --steps 20 --warmup 3 || exit 1
