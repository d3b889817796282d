# round-4 measurement: kernel traces of the split update (config 3, config-5 shard, 8-slab proxies),
# the D = 4 8-slot variant, and the cold-start probe
mkdir -p gpurun_out/t2
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/cold_start_probe.py > gpurun_out/t2/cold.txt 2>&1 || exit 1
cat gpurun_out/t2/cold.txt
for W in "c3|--steps 10 --warmup 3" "c5|--n 62500000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3"; do
  tag=${W%%|*}; args=${W#*|}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t2/tr_$tag -o run -- python3 bench.py --no-cpu --fit-iters 0 $args > gpurun_out/t2/tr_$tag.txt 2>&1 || exit 1
  python3 - gpurun_out/t2/tr_$tag <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:9]:
    print(f'{r["Name"].split("(")[0][:50]:50s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:9.2f}')
PY
done
for LS in 0 1; do
  PCM_D4_LS8=$LS timeout -k 10 200 python bench.py --n 62500000 --k 4096 --d 4 --dtype f16 --no-cpu --fit-iters 0 --steps 10 --warmup 3 > gpurun_out/t2/c5_ls$LS.json 2>&1 || exit 1
  python3 -c "import json;b=json.loads(open('gpurun_out/t2/c5_ls$LS.json').read().strip().splitlines()[-1]);print('c5 LS8=$LS', round(b['ms_per_step'],4), b['breakdown_ms_per_iter'], b['roofline']['kernel'])"
  PCM_D4_LS8=$LS timeout -k 10 300 python bench.py --slab-of 8 --n 500000000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3 > gpurun_out/t2/s8c5_ls$LS.json 2>&1 || exit 1
  python3 -c "import json;b=json.loads(open('gpurun_out/t2/s8c5_ls$LS.json').read().strip().splitlines()[-1]);print('slab8 c5 LS8=$LS', b['value'], b['per_rank_us'])"
done
# D = 4 pruning-grid size (cells per shard) with the 3-level lists
for CT in 20000 32000; do
  PCM_CELL_TARGET=$CT timeout -k 10 200 python bench.py --n 62500000 --k 4096 --d 4 --dtype f16 --no-cpu --fit-iters 0 --steps 10 --warmup 3 > gpurun_out/t2/c5_ct$CT.json 2>&1 || exit 1
  python3 -c "import json;b=json.loads(open('gpurun_out/t2/c5_ct$CT.json').read().strip().splitlines()[-1]);print('c5 cells~$CT', b['config']['grid'], round(b['ms_per_step'],4), b['breakdown_ms_per_iter'], b['candidates']['mean'])"
done
timeout -k 10 200 python bench.py --n 20000000 --k 4096 --clustered 16 --no-cpu --fit-iters 0 --steps 5 --warmup 2 > gpurun_out/t2/cl16.json 2>&1 || exit 1
python3 -c "import json;b=json.loads(open('gpurun_out/t2/cl16.json').read().strip().splitlines()[-1]);print('cl16', round(b['ms_per_step'],4), b['breakdown_ms_per_iter'])"
timeout -k 10 200 python bench.py --no-cpu --fit-iters 20 --steps 20 --warmup 5 > gpurun_out/t2/c3.json 2>&1 || exit 1
python3 -c "import json;b=json.loads(open('gpurun_out/t2/c3.json').read().strip().splitlines()[-1]);print('c3', round(b['ms_per_step'],4), b['breakdown_ms_per_iter'], b['layout_ms'], b['fit'])"
timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > gpurun_out/t2/proxy8.json 2>&1 || exit 1
python3 -c "import json;b=json.loads(open('gpurun_out/t2/proxy8.json').read().strip().splitlines()[-1]);print('proxy8', b['value'], b['per_rank_us'])"
