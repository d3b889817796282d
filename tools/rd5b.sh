#!/bin/bash
# round 5: big tiles + exact grids + one-generation slabs -- parity, bench, 8-slab proxy sweep, rocprof
T=gpurun_out/rd5b; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_crowded.py tests/test_gpu_tiles.py tests/test_gpu_parity.py tests/test_plugin.py tests/test_gpu_baseline_sizes.py -m gpu -x -v --timeout 200 --timeout-method thread > $T/pytest.txt 2>&1; rc=$?
grep -E "passed|failed" $T/pytest.txt | tail -2; grep -E "^(many|clusters) " $T/pytest.txt | cut -c1-300
[ $rc -eq 0 ] || { grep -B5 -A30 "^E " $T/pytest.txt | head -80; exit $rc; }
timeout -k 10 300 python bench.py --fit > $T/bench.json 2>&1 || { tail -20 $T/bench.json; exit 1; }
tail -1 $T/bench.json | cut -c1-300
for F in 0 0.75 0.85 0.95; do
  PCM_ONEGEN_FILL=$F timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > $T/proxy8_$F.json 2>&1 || { tail -20 $T/proxy8_$F.json; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('$T/proxy8_$F.json').read().strip().splitlines()[-1]);s=d['slabs'][0];print('fill $F', round(d['value'],1), d['per_rank_us']['assign'][:3], d['per_rank_us']['step'][:3], s['ncells'], s['ntiles'], round(s['mean'],2), d['centres_bitwise_equal_single_engine'])"
done
bash tools/prof.sh $T/prof --steps 20 --warmup 3 --fit | tail -14 || exit 1
bash tools/prof.sh $T/prof8 --slab-of 8 --steps 20 --warmup 3 | tail -14 || exit 1
