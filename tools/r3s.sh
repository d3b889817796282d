#!/bin/bash
# k_kpp_eval / k_kpp_apply in the late k-means++ steps (last 300 dispatches of a config-3 seeding):
# instruction-fetch waits vs wave cycles
OUT=gpurun_out/r3s; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for P in "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVES SQ_WAVE_CYCLES" "SQ_IFETCH SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY"; do
  n=$(echo $P | tr " " _)
  timeout -k 10 -s KILL 200 rocprofv3 --pmc $P --output-format csv -d $OUT/$n -o run -- python3 tools/kpp_bench.py 100000000 1024 3 > $OUT/$n.log 2>&1 || { echo "FAIL $n"; tail -3 $OUT/$n.log; exit 1; }
  for K in k_kpp_eval k_kpp_apply k_kpp_search; do echo "== $K $n"; PMC_LAST=300 python3 tools/pmc_summary.py $K $OUT/$n/ 2>&1 | tr -d '\n' ; echo; done
done
