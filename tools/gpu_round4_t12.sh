# round-4: compressed-tile prefetch depth (PCM_ZPF 2 = the build, 3, 4: tools/ab/lib_pf*.so):
# parity of the deepest, then alternating config-3 lines and 8-slab proxies
mkdir -p gpurun_out/t12
export PYTHONUNBUFFERED=1
PCM_SO=$GRAFT_REPO_ROOT/tools/ab/lib_pf4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compressed.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t12/pytest.txt 2>&1 || { tail -30 gpurun_out/t12/pytest.txt; exit 1; }
tail -1 gpurun_out/t12/pytest.txt
for i in 1 2; do
  for V in pf2 pf3 pf4; do
    if [ $V = pf2 ]; then unset PCM_SO; else export PCM_SO=$GRAFT_REPO_ROOT/tools/ab/lib_$V.so; fi
    timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 --steps 20 --warmup 3 > gpurun_out/t12/c3_$V$i.json 2>&1 || { tail -5 gpurun_out/t12/c3_$V$i.json; exit 1; }
    python3 -c "import json;b=json.loads(open('gpurun_out/t12/c3_$V$i.json').read().strip().splitlines()[-1]);print('c3 $V$i', round(b['ms_per_step'],4), round(b['roofline']['avg_launch_ms'],4), round(b['roofline']['avg_launch_ms_back_to_back'],4))"
    timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > gpurun_out/t12/p8_$V$i.json 2>&1 || { tail -5 gpurun_out/t12/p8_$V$i.json; exit 1; }
    python3 -c "import json;b=json.loads(open('gpurun_out/t12/p8_$V$i.json').read().strip().splitlines()[-1]);print('p8 $V$i', round(b['value'],2), 'assign', b['per_rank_us']['assign'], 'step', b['per_rank_us']['step'][:2])"
  done
done
