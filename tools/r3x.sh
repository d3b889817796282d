#!/bin/bash
# 8-way slab proxy: per-rank iteration vs points per tile and k_step blocks per coarse cell
T=gpurun_out/r3x; mkdir -p $T
export PYTHONUNBUFFERED=1
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > $T/$name.json 2>&1 || { tail -5 $T/$name.json; exit 1; }
  tail -1 $T/$name.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['per_rank_us']; print('$name', round(d['value'],1), 'assign', max(r['assign']), 'step', max(r['step']), 'kern', d['slabs'][0]['kernel'], 'tiles', d['slabs'][0]['ntiles'])"
}
run base PCM_X=0
run tile3072 PCM_TILE_CAP=3072
run tile2048 PCM_TILE_CAP=2048
run bpc4 PCM_CAND_BPC_RT=4
run bpc16 PCM_CAND_BPC_RT=16
run bpc2 PCM_CAND_BPC_RT=2
