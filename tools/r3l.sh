#!/bin/bash
# crowded instance (CROWD template, LDS long-list words): parity, clustered / uniform timing, slab proxy 8, rocprof
T=gpurun_out/r3l; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_crowded.py tests/test_gpu_compressed.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -60 $T/pytest.txt; exit 1; }
tail -2 $T/pytest.txt
for C in 16 256; do
  timeout -k 10 300 python bench.py --no-cpu --fit-iters 0 --n 20000000 --k 4096 --clustered $C --steps 10 --warmup 3 > $T/clustered$C.txt 2>&1 || { tail -20 $T/clustered$C.txt; exit 1; }
  tail -1 $T/clustered$C.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('clustered $C: ms/it', round(d['ms_per_step'],4), 'brk', d.get('breakdown_ms_per_iter'), 'layout', d.get('layout_ms'), 'kernel', d['roofline']['kernel'], 'cand', d['candidates'])"
done
timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 5 > $T/bench.txt 2>&1 || { tail -20 $T/bench.txt; exit 1; }
tail -1 $T/bench.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('uniform: ms/it', round(d['ms_per_step'],4), 'brk', d.get('breakdown_ms_per_iter'), 'layout', d.get('layout_ms'), 'fit', d.get('fit'))"
timeout -k 10 300 python bench.py --slab-of 8 --steps 20 --warmup 3 > $T/proxy8.json 2>&1 || { tail -20 $T/proxy8.json; exit 1; }
tail -1 $T/proxy8.json | cut -c1-420
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/prof -o run -- python3 bench.py --no-cpu --steps 20 --warmup 5 > $T/prof.log 2>&1 || { tail -20 $T/prof.log; exit 1; }
f=$(find $T/prof -name "*kernel_stats.csv" | head -1); cp $f $T/kernel_stats.csv; head -8 $T/kernel_stats.csv | cut -c1-160
