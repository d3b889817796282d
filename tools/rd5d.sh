#!/bin/bash
# round 5: per-block k_lloyd1 timelines on the 8-way config-4 slab (debug build), default grid vs one generation
T=gpurun_out/rd5d; mkdir -p $T
export PYTHONUNBUFFERED=1
for F in 0 0.9; do
  PCM_ONEGEN_FILL=$F timeout -k 10 200 python tools/lloyd_timing.py tools/ab/lib_dbg.so 10 100000000 1024 3 slab 8 > $T/lt8_$F.txt 2>&1 || { tail -20 $T/lt8_$F.txt; exit 1; }
  cat $T/lt8_$F.txt
done
timeout -k 10 200 python tools/lloyd_timing.py tools/ab/lib_dbg.so 10 > $T/lt_c3.txt 2>&1 || { tail -20 $T/lt_c3.txt; exit 1; }
cat $T/lt_c3.txt
