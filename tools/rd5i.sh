#!/bin/bash
# round 5: persistent prefetching assign (k_lloyd2) -- parity, config-3 and 8-slab A/B against k_lloyd1
T=gpurun_out/rd5i; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py tests/test_gpu_compressed.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread > $T/pytest.txt 2>&1; rc=$?
tail -1 $T/pytest.txt
[ $rc -eq 0 ] || { grep -B5 -A30 "^E " $T/pytest.txt | head -80; exit $rc; }
for V in 1 0 1 0; do
  PCM_LLOYD2=$V timeout -k 10 300 python bench.py --no-cpu --fit-iters 0 > $T/c3_$V.json 2>&1 || { tail -20 $T/c3_$V.json; exit 1; }
  python3 -c "import json;d=json.loads(open('$T/c3_$V.json').read().strip().splitlines()[-1]);print('lloyd2=$V c3', round(d['ms_per_step'],5), {k: round(v,5) for k,v in d['breakdown_ms_per_iter'].items()}, d['roofline']['kernel'], round(d['roofline']['avg_launch_ms_back_to_back'],5))"
  PCM_LLOYD2=$V timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > $T/p8_$V.json 2>&1 || { tail -20 $T/p8_$V.json; exit 1; }
  python3 -c "import json;d=json.loads(open('$T/p8_$V.json').read().strip().splitlines()[-1]);print('lloyd2=$V proxy8', round(d['value'],1), d['per_rank_us']['assign'], d['centres_bitwise_equal_single_engine'])"
done
