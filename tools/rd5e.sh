#!/bin/bash
# round 5: tail split -- parity, 8-slab proxy A/B, per-block timeline, config-3 A/B
T=gpurun_out/rd5e; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiles.py -m gpu -x -q --timeout 200 --timeout-method thread > $T/pytest.txt 2>&1; rc=$?
tail -1 $T/pytest.txt
[ $rc -eq 0 ] || { grep -B5 -A30 "^E " $T/pytest.txt | head -80; exit $rc; }
for F in 0 1 0.5 1.5; do
  PCM_TAIL_SPLIT=$F timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > $T/proxy8_$F.json 2>&1 || { tail -20 $T/proxy8_$F.json; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('$T/proxy8_$F.json').read().strip().splitlines()[-1]);s=d['slabs'][0];print('split $F', round(d['value'],1), d['per_rank_us']['assign'][:4], d['per_rank_us']['step'][:4], s['ncells'], s['ntiles'], round(s['mean'],2), d['centres_bitwise_equal_single_engine'])"
done
PCM_TAIL_SPLIT=1 timeout -k 10 200 python tools/lloyd_timing.py tools/ab/lib_dbg.so 10 100000000 1024 3 slab 8 > $T/lt8.txt 2>&1 || { tail -20 $T/lt8.txt; exit 1; }
head -9 $T/lt8.txt | tail -8
for F in 0 1; do
  PCM_TAIL_SPLIT=$F timeout -k 10 300 python bench.py --no-cpu --fit-iters 0 > $T/c3_$F.json 2>&1 || { tail -20 $T/c3_$F.json; exit 1; }
  python3 -c "import json;d=json.loads(open('$T/c3_$F.json').read().strip().splitlines()[-1]);print('c3 split $F', d['ms_per_step'], d['breakdown_ms_per_iter']['assign'], d['roofline']['avg_launch_ms_back_to_back'], d['config']['tiles'])"
done
PCM_TAIL_SPLIT=0 timeout -k 10 300 python bench.py --no-cpu --fit-iters 0 > $T/c3_0b.json 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('$T/c3_0b.json').read().strip().splitlines()[-1]);print('c3 split 0 again', d['ms_per_step'], d['breakdown_ms_per_iter']['assign'], d['roofline']['avg_launch_ms_back_to_back'])"
