#!/bin/bash
# round 5 baseline: new GPU tests, default bench line, rocprof stats of the bench, 8-slab proxy + its rocprof
T=gpurun_out/rd5a; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_crowded.py tests/test_plugin.py -m gpu -x -v --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1; rc=$?
grep -E "passed|failed" $T/pytest.txt | tail -2; grep -E "^(many|clusters) " $T/pytest.txt | cut -c1-400
[ $rc -eq 0 ] || { grep -B5 -A30 "^E " $T/pytest.txt | head -60; exit $rc; }
timeout -k 10 300 python bench.py --fit > $T/bench.json 2>&1 || { tail -20 $T/bench.json; exit 1; }
tail -1 $T/bench.json | cut -c1-300
bash tools/prof.sh $T/prof --steps 20 --warmup 3 --fit | tail -14 || exit 1
timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > $T/proxy8.json 2>&1 || { tail -20 $T/proxy8.json; exit 1; }
tail -1 $T/proxy8.json | cut -c1-700
bash tools/prof.sh $T/prof8 --slab-of 8 --steps 20 --warmup 3 | tail -14 || exit 1
