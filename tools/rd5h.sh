#!/bin/bash
# round 5: single-GPU iterations through the single statistics buffer -- parity tests, config-3 A/B
T=gpurun_out/rd5h; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py tests/test_gpu_compressed.py tests/test_gpu_crowded.py tests/test_estimator.py tests/test_kpp.py -m gpu -x -q --timeout 300 --timeout-method thread > $T/pytest.txt 2>&1; rc=$?
tail -1 $T/pytest.txt
[ $rc -eq 0 ] || { grep -B5 -A30 "^E " $T/pytest.txt | head -80; exit $rc; }
for P in 1 0 1 0; do
  PCM_PARITY_ITER=$P timeout -k 10 300 python bench.py --no-cpu --fit > $T/c3_$P.json 2>&1 || { tail -20 $T/c3_$P.json; exit 1; }
  python3 -c "import json;d=json.loads(open('$T/c3_$P.json').read().strip().splitlines()[-1]);print('parity $P', round(d['ms_per_step'],5), {k: round(v,5) for k,v in d['breakdown_ms_per_iter'].items()}, 'fit', round(d['fit']['warm_ms'],3), 'kpp', round(d.get('kmeanspp_ms'),1))"
done
