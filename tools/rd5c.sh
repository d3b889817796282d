#!/bin/bash
# round 5: one-generation slab sweep after the sign-mode fix + big-tile parity
T=gpurun_out/rd5c; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiles.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 200 --timeout-method thread > $T/pytest.txt 2>&1; rc=$?
tail -1 $T/pytest.txt
[ $rc -eq 0 ] || { grep -B5 -A30 "^E " $T/pytest.txt | head -80; exit $rc; }
for F in 0 0.8 0.9 1.0; do
  PCM_ONEGEN_FILL=$F timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > $T/proxy8_$F.json 2>&1 || { tail -20 $T/proxy8_$F.json; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('$T/proxy8_$F.json').read().strip().splitlines()[-1]);s=d['slabs'][0];print('fill $F', round(d['value'],1), d['per_rank_us']['assign'][:4], d['per_rank_us']['step'][:4], s['ncells'], s['ntiles'], round(s['mean'],2), d['centres_bitwise_equal_single_engine'])"
done
PCM_ONEGEN_FILL=0.9 bash tools/prof.sh $T/prof8 --slab-of 8 --steps 20 --warmup 3 | tail -6 || exit 1
