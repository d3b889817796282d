#!/bin/bash
# Per-kernel A/B of an environment switch: rocprofv3 kernel stats of the config-3 bench (no k-means++) per value
#   tools/ab_prof.sh OUT VAR "v1 v2" [kernel name patterns...]
set -o pipefail
T=gpurun_out/$1; VAR=$2; VALS=$3; shift 3; mkdir -p $T
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in $VALS; do
  t=${v//\//_}
  env $VAR=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $T/p_$t -o run -- python3 bench.py --no-cpu --no-kpp --steps 20 > $T/b_$t.json 2> $T/b_$t.err || { tail -20 $T/b_$t.err; exit 1; }
  f=$(ls $T/p_$t/*/run_kernel_stats.csv $T/p_$t/run_kernel_stats.csv 2>/dev/null | head -1)
  python3 - "$f" "$VAR=$v" "$@" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
pats = sys.argv[3:] or ["k_rs_", "k_lloyd1", "k_lab_gather", "k_updlists", "k_label"]
for r in rows:
    if any(p in r["Name"] for p in pats):
        print(sys.argv[2].split("/")[-1], r["Name"].split("(")[0][:60], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 1))
PY
  tail -1 $T/b_$t.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', 'layout', round(d['layout_ms'],3), 'fit warm', round(d['fit']['warm_ms'],3))"
done
