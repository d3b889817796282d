# round-4: cold start on a fresh box (first GPU process), tests, crowded-cloud and
# config-5 counter sets, bench lines
mkdir -p gpurun_out/t4
export PYTHONUNBUFFERED=1
timeout -k 10 120 python tools/cold_start_probe.py > gpurun_out/t4/cold.txt 2>&1 || exit 1
cat gpurun_out/t4/cold.txt
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t4/pytest.txt 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/t4/pytest.txt | tail -5
[ $rc -eq 0 ] || { grep -B5 -A30 "^E " gpurun_out/t4/pytest.txt | head -60; exit $rc; }
for W in "c3|--steps 20 --warmup 5" "c5|--n 62500000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3"; do
  tag=${W%%|*}; args=${W#*|}
  timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 $args > gpurun_out/t4/$tag.json 2>&1 || exit 1
  python3 -c "import json;b=json.loads(open('gpurun_out/t4/$tag.json').read().strip().splitlines()[-1]);print('$tag', round(b['ms_per_step'],4), b['breakdown_ms_per_iter'], round(b['roofline']['frac'],3), b['roofline']['kernel'])"
done
timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > gpurun_out/t4/proxy8.json 2>&1 || exit 1
python3 -c "import json;b=json.loads(open('gpurun_out/t4/proxy8.json').read().strip().splitlines()[-1]);print('proxy8', b['value'], b['per_rank_us'])"
timeout -k 10 300 python bench.py --slab-of 8 --n 500000000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3 > gpurun_out/t4/s8c5.json 2>&1 || exit 1
python3 -c "import json;b=json.loads(open('gpurun_out/t4/s8c5.json').read().strip().splitlines()[-1]);print('slab8 c5', b['value'], b['per_rank_us'])"
bash tools/kernel_profile.sh gpurun_out/t4/pc_cl16 k_lloyd1 --n 20000000 --k 4096 --clustered 16 --steps 5 --warmup 2 > gpurun_out/t4/pc_cl16.txt 2>&1 || { tail -5 gpurun_out/t4/pc_cl16.txt; exit 1; }
tail -42 gpurun_out/t4/pc_cl16.txt | grep -E "k_lloyd1|k_tile|k_cand|k_lists|SQ_|clock|frac|hbm|_ns"
bash tools/kernel_profile.sh gpurun_out/t4/pc_c5 k_lloyd1 --n 62500000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3 > gpurun_out/t4/pc_c5.txt 2>&1 || { tail -5 gpurun_out/t4/pc_c5.txt; exit 1; }
tail -42 gpurun_out/t4/pc_c5.txt | grep -E "SQ_|clock|frac|hbm|_ns"
