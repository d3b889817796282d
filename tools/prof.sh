#!/bin/bash
# rocprofv3 kernel-trace stats of the headline bench (GPU box): tools/prof.sh OUTDIR [bench args]
OUT=$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu "$@" > $OUT/bench.txt 2>&1 || { tail -20 $OUT/bench.txt; exit 1; }
tail -1 $OUT/bench.txt
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:12]:
    print(f'{r["Name"][:70]:70s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:9.2f} pct={r["Percentage"]}')
PY
