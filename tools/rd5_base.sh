#!/bin/bash
# round 5 baseline: default bench line, rocprof stats of the bench, 8-slab proxies (config 4 and 5)
T=gpurun_out/rd5a; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --fit > $T/bench.json 2>&1 || { tail -20 $T/bench.json; exit 1; }
tail -1 $T/bench.json | cut -c1-600
bash tools/prof.sh $T/prof --steps 20 --warmup 3 --fit | tail -14 || exit 1
timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > $T/proxy8.json 2>&1 || { tail -20 $T/proxy8.json; exit 1; }
tail -1 $T/proxy8.json | cut -c1-900
bash tools/prof.sh $T/prof8 --slab-of 8 --steps 20 --warmup 3 | tail -14 || exit 1
