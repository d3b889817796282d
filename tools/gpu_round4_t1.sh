mkdir -p gpurun_out/t1
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t1/pytest.txt 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/t1/pytest.txt | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu --fit-iters 20 --steps 20 --warmup 5 > gpurun_out/t1/c3.json 2>&1 || exit 1
tail -c 900 gpurun_out/t1/c3.json
timeout -k 10 200 python bench.py --n 62500000 --k 4096 --d 4 --dtype f16 --no-cpu --fit-iters 0 --steps 10 --warmup 3 > gpurun_out/t1/c5.json 2>&1 || exit 1
tail -c 600 gpurun_out/t1/c5.json
timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > gpurun_out/t1/proxy8.json 2>&1 || exit 1
python3 -c "import json;b=json.loads(open('gpurun_out/t1/proxy8.json').read().strip().splitlines()[-1]);print(b['value'],b['per_rank_us'],b['centres_bitwise_equal_single_engine'])"
timeout -k 10 200 python bench.py --n 20000000 --k 4096 --clustered 16 --no-cpu --fit-iters 0 --steps 5 --warmup 2 > gpurun_out/t1/cl16.json 2>&1 || exit 1
tail -c 700 gpurun_out/t1/cl16.json
