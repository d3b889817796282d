#!/bin/bash
# GPU tests + short bench (used from gpurun): tools/gt.sh [bench args]
mkdir -p gpurun_out/gt
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/gt/pytest.txt 2>&1
rc=$?; tail -15 gpurun_out/gt/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 3 "$@" > gpurun_out/gt/bench.txt 2>&1 || { tail -20 gpurun_out/gt/bench.txt; exit 1; }
tail -1 gpurun_out/gt/bench.txt
