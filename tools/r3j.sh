#!/bin/bash
# crowded layouts (Morton-ordered cells + tile lists): parity, then clustered / uniform re-time
T=gpurun_out/r3j; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_crowded.py -m gpu -x -v --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -60 $T/pytest.txt; exit 1; }
tail -3 $T/pytest.txt
for C in 16 256; do
  timeout -k 10 300 python bench.py --no-cpu --fit-iters 0 --n 20000000 --k 4096 --clustered $C --steps 10 --warmup 3 > $T/clustered$C.txt 2>&1 || { tail -20 $T/clustered$C.txt; exit 1; }
  tail -1 $T/clustered$C.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('clustered $C: ms/it', round(d['ms_per_step'],4), 'assign', round(d['roofline']['avg_launch_ms'],4), 'brk', d.get('breakdown_ms_per_iter'), 'layout', d.get('layout_ms'), 'cand', d['candidates'])"
done
timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 5 > $T/bench.txt 2>&1 || { tail -20 $T/bench.txt; exit 1; }
tail -1 $T/bench.txt | cut -c1-700
