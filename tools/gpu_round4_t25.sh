# round-4: the multi-GPU call sequence on one GPU through RCCL (an nccl group of 1, graph capture of
# k_lloyd1 + all-reduce + k_updlists), config-4 slab size and config 3; gloo 2-rank rehearsal of config 5
mkdir -p gpurun_out/t25
export PYTHONUNBUFFERED=1
timeout -k 10 200 python bench.py --split --n 12500000 --no-cpu --fit-iters 0 --steps 20 --warmup 3 > gpurun_out/t25/split12.json 2>&1 || { tail -8 gpurun_out/t25/split12.json; exit 1; }
python3 -c "import json;b=json.loads(open('gpurun_out/t25/split12.json').read().strip().splitlines()[-1]);print('split 12.5M', b['ms_per_step'], b['config']['launch'], b.get('graph_error'), b['breakdown_ms_per_iter'])"
timeout -k 10 200 python bench.py --split --no-cpu --fit-iters 0 --steps 20 --warmup 3 > gpurun_out/t25/split100.json 2>&1 || { tail -8 gpurun_out/t25/split100.json; exit 1; }
python3 -c "import json;b=json.loads(open('gpurun_out/t25/split100.json').read().strip().splitlines()[-1]);print('split 100M', b['ms_per_step'], b['config']['launch'], b.get('graph_error'), b['breakdown_ms_per_iter'])"
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --n 40000000 --k 4096 --d 4 --dtype f16 --no-cpu --fit-iters 0 --steps 3 --warmup 2 > gpurun_out/t25/gloo2_c5.txt 2>&1 || { tail -8 gpurun_out/t25/gloo2_c5.txt; exit 1; }
tail -1 gpurun_out/t25/gloo2_c5.txt | cut -c1-300
