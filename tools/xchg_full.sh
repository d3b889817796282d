#!/bin/bash
# multi-process exchange at full size: 2/3-rank tests, configs 4/5 over 8 gloo ranks on one GPU, bench rehearsal
set -o pipefail
T=gpurun_out/${1:-xf}; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v --timeout 150 --timeout-method thread > $T/pytest_multirank.txt 2>&1 || { tail -40 $T/pytest_multirank.txt; exit 1; }
tail -1 $T/pytest_multirank.txt
timeout -k 10 700 python -u -m pytest tests/test_gpu_full_configs.py -m gpu -x -v --timeout 400 --timeout-method thread > $T/pytest_full.txt 2>&1 || { tail -40 $T/pytest_full.txt; exit 1; }
tail -4 $T/pytest_full.txt
timeout -k 10 200 python bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 --no-cpu --fit-iters 0 > $T/bench_gloo2.json 2> $T/bench_gloo2.err || { tail -20 $T/bench_gloo2.err; exit 1; }
tail -1 $T/bench_gloo2.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['config']['exchange'], d['config']['launch'], d['breakdown_ms_per_iter'])"
