#!/bin/bash
# k-means++ late-grid divisor after the atomics fix (eval/apply blocks from centre 64 on = 2048 / DIV)
T=gpurun_out/r4j; mkdir -p $T
export PYTHONUNBUFFERED=1
for DIV in 4 2 8 4; do
  PCM_KPP_LATE_DIV=$DIV timeout -k 10 200 python tools/kpp_bench.py 100000000 1024 3 > $T/kpp_$DIV.txt 2>&1 || { tail -5 $T/kpp_$DIV.txt; exit 1; }
  echo "div=$DIV: $(grep 'call 1' $T/kpp_$DIV.txt)"
done
