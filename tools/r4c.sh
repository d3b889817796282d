#!/bin/bash
# full GPU suite; k-means++ dense threshold 7/8; slab proxies with one k_step block per CU on fine grids
T=gpurun_out/r4c; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -60 $T/pytest.txt; exit 1; }
tail -1 $T/pytest.txt
timeout -k 10 300 bash tools/kpp_prof.sh r4c_prof > $T/kpp_prof.txt 2>&1 || { tail -20 $T/kpp_prof.txt; exit 1; }
tail -5 $T/kpp_prof.txt
for P in 2 4 8; do
  timeout -k 10 200 python bench.py --slab-of $P --steps 20 --warmup 3 > $T/proxy$P.json 2>&1 || { tail -20 $T/proxy$P.json; exit 1; }
  tail -1 $T/proxy$P.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['per_rank_us']; print('P=$P', round(d['value'],1), 'assign', r['assign'], 'step', r['step'])"
done
for V in prod rs512; do
  SO=""; [ $V = rs512 ] && SO=tools/variants/lib_rs512.so
  PCM_SO=$SO timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 3 > $T/bench_$V.txt 2>&1 || { tail -20 $T/bench_$V.txt; exit 1; }
  tail -1 $T/bench_$V.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$V ms/it', round(d['ms_per_step'],4), 'layout', d.get('layout_ms'), 'fit', d.get('fit'))"
done
PCM_SO=tools/variants/lib_rs512.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest_rs512.txt 2>&1 || { tail -30 $T/pytest_rs512.txt; exit 1; }
tail -1 $T/pytest_rs512.txt
