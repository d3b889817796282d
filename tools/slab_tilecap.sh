#!/bin/bash
# 8-slab proxy vs tile cap (PCM_TILE_CAP) and the longest-list-first order (PCM_TILE_LPT), alternating
mkdir -p gpurun_out/slabcap
for r in 1 2; do for cfg in "4096 -1" "3072 1" "2048 1" "2048 0"; do set -- $cfg
  PCM_TILE_CAP=$1 PCM_TILE_LPT=$2 timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > gpurun_out/slabcap/s8_$1_$2_$r.json 2>&1 || { tail -5 gpurun_out/slabcap/s8_$1_$2_$r.json; exit 1; }
  tail -1 gpurun_out/slabcap/s8_$1_$2_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cap $1 lpt $2', 'us/rank', round(d['value'],1), 'assign max', max(d['per_rank_us']['assign']), 'tiles', d['slabs'][0]['ntiles'], 'bitwise', d['centres_bitwise_equal_single_engine'])"
done; done
