#!/bin/bash
# k-means++ grid sweep after the atomics fix: eval/apply blocks from centre LATE_C on = pgrid / LATE_DIV
T=gpurun_out/r3v; mkdir -p $T
export PYTHONUNBUFFERED=1
for cfg in "4 64" "2 64" "1 64" "2 300" "1 300"; do
  set -- $cfg
  PCM_KPP_LATE_DIV=$1 PCM_KPP_LATE_C=$2 timeout -k 10 200 python tools/kpp_bench.py 100000000 1024 3 > $T/kpp_$1_$2.txt 2>&1 || { tail -5 $T/kpp_$1_$2.txt; exit 1; }
  echo "div=$1 c=$2: $(grep 'call 1' $T/kpp_$1_$2.txt)"
done
