#!/bin/bash
# k-means++ two-cells-per-pass: parity, per-step means, late-grid sweep
T=gpurun_out/r3w; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -60 $T/pytest.txt; exit 1; }
tail -1 $T/pytest.txt
timeout -k 10 300 bash tools/kpp_prof.sh r3w_prof > $T/kpp_prof.txt 2>&1 || { tail -20 $T/kpp_prof.txt; exit 1; }
tail -5 $T/kpp_prof.txt
for cfg in "2 64" "1 64" "2 300"; do
  set -- $cfg
  PCM_KPP_LATE_DIV=$1 PCM_KPP_LATE_C=$2 timeout -k 10 200 python tools/kpp_bench.py 100000000 1024 3 > $T/kpp_$1_$2.txt 2>&1 || { tail -5 $T/kpp_$1_$2.txt; exit 1; }
  echo "div=$1 c=$2: $(grep 'call 1' $T/kpp_$1_$2.txt)"
done
