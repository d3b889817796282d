#!/bin/bash
# round 3 check: slab-sharded multirank tests, 1-GPU slab proxy, gloo rehearsal of bench --gpus 2
T=gpurun_out/r3a; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py tests/test_plugin_cloud_golden.py tests/test_stages_reference.py -m gpu -x -v --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -40 $T/pytest.txt; exit 1; }
tail -2 $T/pytest.txt
timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > $T/proxy8.txt 2>&1 || { tail -20 $T/proxy8.txt; exit 1; }
tail -1 $T/proxy8.txt
for P in 2 4; do timeout -k 10 200 python bench.py --slab-of $P --steps 20 --warmup 3 > $T/proxy$P.txt 2>&1 || { tail -20 $T/proxy$P.txt; exit 1; }; tail -1 $T/proxy$P.txt; done
timeout -k 10 200 python bench.py --split --no-cpu --fit-iters 0 --steps 20 --warmup 3 --n 12500000 > $T/rows12p5.txt 2>&1 || { tail -20 $T/rows12p5.txt; exit 1; }
tail -1 $T/rows12p5.txt
timeout -k 10 200 python bench.py --gpus 2 --backend gloo --n 20000000 --no-cpu --fit-iters 0 --steps 5 --warmup 2 > $T/gloo2.txt 2>&1 || { tail -20 $T/gloo2.txt; exit 1; }
tail -1 $T/gloo2.txt
timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 3 > $T/bench1.txt 2>&1 || { tail -20 $T/bench1.txt; exit 1; }
tail -1 $T/bench1.txt
