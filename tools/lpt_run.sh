export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compressed.py tests/test_gpu_xchg.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lpt2_pytest.txt 2>&1 || { tail -30 gpurun_out/lpt2_pytest.txt; exit 1; }
tail -1 gpurun_out/lpt2_pytest.txt
bash tools/ab_c5.sh lpt2 PCM_TILE_LPT "0 -1" 2 || exit 1
for v in 0 -1 0 -1; do
  PCM_TILE_LPT=$v timeout -k 10 200 python bench.py --split --no-cpu --fit-iters 0 --n 12500000 > gpurun_out/lpt2/split_$v.json 2>&1 || { tail -5 gpurun_out/lpt2/split_$v.json; exit 1; }
  tail -1 gpurun_out/lpt2/split_$v.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('split12.5M LPT=$v', round(d['ms_per_step']*1e3,1), d['breakdown_ms_per_iter']['assign'])"
done
bash tools/ab_env.sh lpt2c3 PCM_TILE_LPT "0 -1" 2
