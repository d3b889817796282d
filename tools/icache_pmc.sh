#!/bin/bash
# instruction-cache counters of the k-means++ and Lloyd kernels (one --pmc pass each group)
OUT=gpurun_out/${1:-ic}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INSTS_SALU\b" $OUT/avail.txt | sort -u | head -20
for P in "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVES SQ_WAVE_CYCLES" "SQ_IFETCH SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU"; do
  n=$(echo $P | tr " " _)
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/$n -o run -- python3 tools/kpp_bench.py 20000000 512 3 > $OUT/$n.log 2>&1 || { echo "FAIL $n"; tail -3 $OUT/$n.log; continue; }
  python3 tools/pmc_summary.py k_kpp_search $OUT/$n/ 2>&1 | tail -8
  python3 tools/pmc_summary.py k_kpp_eval $OUT/$n/ 2>&1 | tail -8
done
