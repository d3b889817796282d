# round-4: pruning-grid size on the 8-way slabs (PCM_CELL_TARGET; the slab engines' default
# is 32 cells per centre scaled by the slab's share of the cloud): config-5 and config-4 slabs
mkdir -p gpurun_out/t19
export PYTHONUNBUFFERED=1
for T in 16384 32768 62500 16384; do
  PCM_CELL_TARGET=$T timeout -k 10 300 python bench.py --slab-of 8 --n 500000000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3 > gpurun_out/t19/c5_$T.json 2>&1 || { tail -5 gpurun_out/t19/c5_$T.json; exit 1; }
  python3 -c "import json;b=json.loads(open('gpurun_out/t19/c5_$T.json').read().strip().splitlines()[-1]);s=b['slabs'][1];print('c5 slab8 target $T', round(b['value'],1), 'assign', b['per_rank_us']['assign'][1:3], 'step', b['per_rank_us']['step'][1:3], 'cells', s['ncells'], 'tiles', s['ntiles'], 'lists', round(s['mean'],2), s['max'])"
done
for T in 4096 8192 2048 4096; do
  PCM_CELL_TARGET=$T timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > gpurun_out/t19/c4_$T.json 2>&1 || { tail -5 gpurun_out/t19/c4_$T.json; exit 1; }
  python3 -c "import json;b=json.loads(open('gpurun_out/t19/c4_$T.json').read().strip().splitlines()[-1]);s=b['slabs'][1];print('c4 slab8 target $T', round(b['value'],1), 'assign', b['per_rank_us']['assign'][1:3], 'step', b['per_rank_us']['step'][1:3], 'cells', s['ncells'], 'tiles', s['ntiles'], 'lists', round(s['mean'],2), s['max'])"
done
