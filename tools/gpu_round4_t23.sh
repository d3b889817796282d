# round-4: config-5 slab grid size again with the 256-thread mid-cell list blocks
mkdir -p gpurun_out/t23
export PYTHONUNBUFFERED=1
for T in 16384 24576 32768 16384 24576 32768; do
  PCM_CELL_TARGET=$T timeout -k 10 300 python bench.py --slab-of 8 --n 500000000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3 > gpurun_out/t23/c5_$T.json 2>&1 || { tail -5 gpurun_out/t23/c5_$T.json; exit 1; }
  python3 -c "import json;b=json.loads(open('gpurun_out/t23/c5_$T.json').read().strip().splitlines()[-1]);s=b['slabs'][1];print('c5 slab8 target $T', round(b['value'],1), 'assign', b['per_rank_us']['assign'][1:3], 'step', b['per_rank_us']['step'][1:3], 'cells', s['ncells'], 'tiles', s['ntiles'], 'lists', round(s['mean'],2), s['max'])"
done
