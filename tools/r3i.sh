#!/bin/bash
# FULL-tile scan with batched scalar loads: parity (compressed + clustered tests), clustered re-time, config-5 proxy
T=gpurun_out/r3i; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_compressed.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -40 $T/pytest.txt; exit 1; }
tail -3 $T/pytest.txt
for C in 16 256; do
  timeout -k 10 300 python bench.py --no-cpu --fit-iters 0 --n 20000000 --k 4096 --clustered $C --steps 10 --warmup 3 > $T/clustered$C.txt 2>&1 || { tail -20 $T/clustered$C.txt; exit 1; }
  tail -1 $T/clustered$C.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('clustered $C: ms/it', round(d['ms_per_step'],4), 'assign', round(d['roofline']['avg_launch_ms'],4), 'cand', d['candidates'])"
done
echo "== config-5 shape, 8-way slab proxy (fp16, D=4, K=4096, N=500M)"
timeout -k 10 400 python bench.py --slab-of 8 --n 500000000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3 > $T/proxy8_c5.json 2>&1 || { tail -20 $T/proxy8_c5.json; exit 1; }
tail -1 $T/proxy8_c5.json | cut -c1-900
