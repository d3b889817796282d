#!/bin/bash
# A/B of a k_lloyd1 variant library against the product build: parity subset with the variant, then the
# 8-slab proxy (config 4, collective) and the config-3 bench line, alternating
# usage: tools/ab_tpb.sh OUT VARIANT_SO
set -o pipefail
T=gpurun_out/${1:-ab}; V=$2; mkdir -p $T
export PYTHONUNBUFFERED=1
PCM_SO=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py -m gpu -x -q --timeout 200 --timeout-method thread > $T/pytest_variant.txt 2>&1 || { tail -30 $T/pytest_variant.txt; exit 1; }
tail -1 $T/pytest_variant.txt
for rep in 1 2; do for so in default $V; do
  if [ $so = default ]; then unset PCM_SO; else export PCM_SO=$so; fi
  timeout -k 10 200 python bench.py --slab-of 8 --exchange collective --steps 30 --warmup 5 > $T/p8_$(basename $so)_$rep.json 2> $T/p8.err || { tail -20 $T/p8.err; exit 1; }
  python -c "import json; d=json.loads(open('$T/p8_$(basename $so)_$rep.json').read().strip().splitlines()[-1]); print('p8', '$(basename $so)', round(d['value'],2), d['per_rank_us']['assign'], d['centres_bitwise_equal_single_engine'])"
  timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 --no-kpp --steps 20 > $T/c3_$(basename $so)_$rep.json 2> $T/c3.err || { tail -20 $T/c3.err; exit 1; }
  python -c "import json; d=json.loads(open('$T/c3_$(basename $so)_$rep.json').read().strip().splitlines()[-1]); print('c3', '$(basename $so)', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
done; done
unset PCM_SO
