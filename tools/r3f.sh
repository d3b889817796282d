#!/bin/bash
# round 3: compressed point stream -- full GPU parity, A/B (PCM_XZ=0/1), rocprof stats, slab proxy
T=gpurun_out/r3f; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -40 $T/pytest.txt; exit 1; }
tail -2 $T/pytest.txt
for Z in 1 0; do
  PCM_XZ=$Z timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 3 > $T/bench_xz$Z.txt 2>&1 || { tail -20 $T/bench_xz$Z.txt; exit 1; }
  tail -1 $T/bench_xz$Z.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('xz=$Z ms/it', round(d['ms_per_step'],4), 'value %.4g' % d['value'], 'assign_ms', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],3), 'B/pt', round(r['algorithmic_bytes_per_point'],2), 'layout', round(d['layout_ms'],2), 'fit', round(d['fit']['warm_ms'],2))"
done
timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > $T/proxy8.txt 2>&1 || { tail -20 $T/proxy8.txt; exit 1; }
tail -1 $T/proxy8.txt | cut -c1-700
bash tools/prof.sh $T/prof --steps 20 --warmup 3 || exit 1
