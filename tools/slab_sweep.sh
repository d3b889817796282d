#!/bin/bash
# per-rank cost of the 8-way slab proxy vs grid density and candidate blocks per coarse cell
T=gpurun_out/slab_sweep; mkdir -p $T
for CT in 0 2048 8192 16384; do
  for BPC in 0 4 16; do
    E=""; [ $CT -gt 0 ] && E="PCM_CELL_TARGET=$CT"; [ $BPC -gt 0 ] && E="$E PCM_CAND_BPC_RT=$BPC"
    env $E timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > $T/ct${CT}_b${BPC}.json 2>&1 || { tail -5 $T/ct${CT}_b${BPC}.json; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('$T/ct${CT}_b${BPC}.json').read().splitlines()[-1]); p=d['per_rank_us']
print('cells=$CT bpc=$BPC max %.1f  assign %.1f..%.1f step %.1f..%.1f ncells %d lists %.2f' % (d['value'], min(p['assign']), max(p['assign']), min(p['step']), max(p['step']), d['slabs'][1]['ncells'], d['slabs'][1]['mean']))"
  done
done
