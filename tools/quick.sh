#!/bin/bash
# quick: parity file(s) + bench lines with the whole-fit timing (config 3) + 12.5M split
set -o pipefail
T=gpurun_out/${1:-q}; shift; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest ${@:-tests/test_gpu_parity.py} -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -30 $T/pytest.txt; exit 1; }
tail -1 $T/pytest.txt
timeout -k 10 200 python bench.py --no-cpu --fit > $T/bench.txt 2>&1 || { tail -20 $T/bench.txt; exit 1; }
tail -1 $T/bench.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['ms_per_step'], d['breakdown_ms_per_iter'], d['roofline']['frac'], 'layout', d['layout_ms'], 'fit', d['fit'], 'kpp', d.get('kmeanspp_ms'))"
timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 --split --n 12500000 > $T/split.txt 2>&1 || { tail -20 $T/split.txt; exit 1; }
tail -1 $T/split.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('s12', d['ms_per_step'], d['breakdown_ms_per_iter'], d['roofline']['frac'])"
