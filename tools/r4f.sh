#!/bin/bash
# calibration: k_lloyd1 with its flush atomics issued twice vs the product (config 3 bench, rocprof)
T=gpurun_out/r4f; mkdir -p $T
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for V in prod dflush prod2; do
  SO=""; [ $V = dflush ] && SO=tools/variants/lib_dflush.so
  PCM_SO=$SO timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/$V -o run -- python3 bench.py --no-cpu --fit-iters 0 --steps 20 --warmup 3 > $T/$V.log 2>&1 || { tail -20 $T/$V.log; exit 1; }
  f=$(find $T/$V -name "*kernel_stats.csv" | head -1)
  echo "$V: $(grep 'k_lloyd1' $f | cut -d, -f2-4)"
done
