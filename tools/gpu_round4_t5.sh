# round-4: candidate-list reuse budget (PCM_DRIFT_KAPPA, cell widths) at the config-5 shard,
# the config-5 8-way slab and the config-4 8-way slab
mkdir -p gpurun_out/t5
export PYTHONUNBUFFERED=1
for KP in 0.05 0.2 0.5 1.0; do
  PCM_DRIFT_KAPPA=$KP timeout -k 10 200 python bench.py --n 62500000 --k 4096 --d 4 --dtype f16 --no-cpu --fit-iters 0 --steps 20 --warmup 3 > gpurun_out/t5/c5_k$KP.json 2>&1 || exit 1
  python3 -c "import json;b=json.loads(open('gpurun_out/t5/c5_k$KP.json').read().strip().splitlines()[-1]);print('c5 kappa $KP', round(b['ms_per_step'],4), b['breakdown_ms_per_iter'], b['candidates'])"
  PCM_DRIFT_KAPPA=$KP timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > gpurun_out/t5/p8_k$KP.json 2>&1 || exit 1
  python3 -c "import json;b=json.loads(open('gpurun_out/t5/p8_k$KP.json').read().strip().splitlines()[-1]);print('proxy8 kappa $KP', b['value'], b['per_rank_us']['assign'][:3], b['per_rank_us']['step'][:3])"
done
