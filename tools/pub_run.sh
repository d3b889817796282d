#!/bin/bash
# k_updlists dedicated publisher (PCM_UPD_PUB): parity subset, then the 8-slab proxy and config 3 A/B
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/pub
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_xchg.py tests/test_gpu_multirank.py tests/test_gpu_crowded.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pub/pytest.txt 2>&1 || { tail -30 gpurun_out/pub/pytest.txt; exit 1; }
tail -1 gpurun_out/pub/pytest.txt
for r in 1 2; do for v in 0 1; do
  PCM_UPD_PUB=$v timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > gpurun_out/pub/s8_${v}_$r.json 2>&1 || { tail -5 gpurun_out/pub/s8_${v}_$r.json; exit 1; }
  tail -1 gpurun_out/pub/s8_${v}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('slab8 PUB=$v', 'us/rank', round(d['value'],1), 'step', d['per_rank_us']['step'], 'bitwise', d['centres_bitwise_equal_single_engine'])"
done; done
bash tools/prof_proxy.sh pub/prof_pub1 --exchange peer || exit 1
