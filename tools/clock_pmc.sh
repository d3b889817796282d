#!/bin/bash
# Effective clock per k_lloyd1 / k_step dispatch (MI355X_MICROARCH.md "DVFS give-back":
# GRBM_GUI_ACTIVE / 8 / kernel wall time) + HBM traffic of the compressed stream.
# usage: tools/clock_pmc.sh OUTDIR [bench args]
OUT=$1; shift; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/clk -o run -- python3 bench.py --no-cpu --fit-iters 0 "$@" > $OUT/clk.txt 2>&1 || { tail -5 $OUT/clk.txt; exit 1; }
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc_$P -o run -- python3 bench.py --no-cpu --no-graph --fit-iters 0 "$@" > $OUT/pmc_$P.log 2>&1 || { echo "FAIL pmc $P"; tail -5 $OUT/pmc_$P.log; exit 1; }
done
python3 tools/pmc_summary.py k_lloyd1 $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE > $OUT/pmc_k_lloyd.json && cat $OUT/pmc_k_lloyd.json
python3 - $OUT <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/clk/**/*counter_collection.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f))]
out = []
for r in rows:
    n = r["Kernel_Name"]
    if "k_lloyd1" not in n and "k_step" not in n:
        continue
    ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) if "End_Timestamp" in r else None
    v = float(r["Counter_Value"])
    out.append(("L" if "k_lloyd1" in n else "S", ns, v))
for k, ns, v in out:
    if ns:
        print(k, round(ns / 1e3, 1), "us", "clk %.2f GHz" % (v / 8 / ns))
PY
