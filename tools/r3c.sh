#!/bin/bash
# round 3: full GPU suite (slab sharding, counting-sort layout, plugin-cloud goldens), slab proxies,
# gloo rehearsal of bench --gpus 2, layout A/B (radix vs counting sort), rocprof kernel stats
T=gpurun_out/r3c; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -40 $T/pytest.txt; exit 1; }
tail -2 $T/pytest.txt
for P in 8 4 2; do timeout -k 10 200 python bench.py --slab-of $P --steps 20 --warmup 3 > $T/proxy$P.txt 2>&1 || { tail -20 $T/proxy$P.txt; exit 1; }; tail -1 $T/proxy$P.txt | cut -c1-600; done
timeout -k 10 200 python bench.py --gpus 2 --backend gloo --n 20000000 --no-cpu --fit-iters 0 --steps 5 --warmup 2 > $T/gloo2.txt 2>&1 || { tail -20 $T/gloo2.txt; exit 1; }
tail -1 $T/gloo2.txt | cut -c1-400
for L in 0 1; do
  PCM_LAYOUT_RADIX=$L timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 3 > $T/bench_radix$L.txt 2>&1 || { tail -20 $T/bench_radix$L.txt; exit 1; }
  tail -1 $T/bench_radix$L.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('radix=$L', 'layout_ms', round(d['layout_ms'],2), 'fit', d['fit'], 'ms/it', round(d['ms_per_step'],4))"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof -o run -- python3 bench.py --no-cpu --steps 20 --warmup 3 > $T/prof.log 2>&1 || { tail -20 $T/prof.log; exit 1; }
find $T/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $T/kernel_stats.csv
head -25 $T/kernel_stats.csv | cut -c1-160
