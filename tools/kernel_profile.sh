#!/bin/bash
# One workload's evidence set on the GPU box:
#   tools/kernel_profile.sh OUT KERNEL_SUBSTR [bench args]
# -> OUT/bench.json      the bench line (no CPU leg, no whole fit)
#    OUT/kernel_stats.csv rocprofv3 --kernel-trace --stats of the same command
#    OUT/pmc.json         per-dispatch means of SQ / TCC / GRBM counters for KERNEL_SUBSTR
#                         (one rocprofv3 --pmc pass per group, eager launches; FETCH_SIZE x2 per
#                         the gfx950 correction; clock_GHz = GRBM_GUI_ACTIVE / 8 / dispatch time)
OUT=$1; KER=$2; shift 2
mkdir -p $OUT
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 bench.py --no-cpu --fit-iters 0 "$@" > $OUT/bench.txt 2>&1 || { tail -20 $OUT/bench.txt; exit 1; }
tail -1 $OUT/bench.txt > $OUT/bench.json
cut -c1-600 $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu --fit-iters 0 "$@" > $OUT/trace.txt 2>&1 || { tail -20 $OUT/trace.txt; exit 1; }
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:10]:
    print(f'{r["Name"][:60]:60s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:9.2f} pct={r["Percentage"]}')
PY
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_VALU_MFMA_BUSY_CYCLES FETCH_SIZE" \
         "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py --no-cpu --fit-iters 0 --no-graph "$@" > $OUT/pmc$i.log 2>&1 || { echo "FAIL pmc pass $i"; tail -5 $OUT/pmc$i.log; exit 1; }
done
python3 tools/pmc_summary.py "$KER" $OUT/pmc1 $OUT/pmc2 $OUT/pmc3 $OUT/pmc4 > $OUT/pmc.json && cat $OUT/pmc.json
