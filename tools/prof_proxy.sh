#!/bin/bash
# rocprofv3 kernel trace of the 8-slab proxy with the peer exchange: per-kernel durations and gaps
# usage: tools/prof_proxy.sh OUT [bench args]
OUT=gpurun_out/$1; shift; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PCM_PROXY_NOCHECK=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --slab-of 8 --steps 40 --warmup 5 "$@" > $OUT/bench.txt 2>&1 || { tail -20 $OUT/bench.txt; exit 1; }
tail -1 $OUT/bench.txt | cut -c1-300
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:12]:
    print(f'{r["Name"][:60]:60s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:8.2f} min_us={float(r["MinNs"])/1e3:8.2f} pct={r["Percentage"]}')
PY
t=$(find $OUT/trace -name "*kernel_trace.csv" | head -1); [ -n "$t" ] && python3 tools/trace_gaps.py $(dirname $t) 240 2>&1 | tail -12
