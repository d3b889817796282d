#!/bin/bash
set -o pipefail
T=gpurun_out/${1:-st}; mkdir -p $T
for v in dbgt; do
for cfg in "s12 12500000 1024 3" "c3 100000000 1024 3"; do
  set -- $cfg
  timeout -k 10 120 python tools/step_timing2.py $PWD/tools/variants/lib_$v.so 10 $2 $3 $4 > $T/st_${v}_$1.txt 2>&1 || { tail -5 $T/st_${v}_$1.txt; exit 1; }
  echo "== $v $1"; grep -v amdgpu.ids $T/st_${v}_$1.txt | grep -v "block start\|slowest\|coarse-list"
done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -30 $T/pytest.txt; exit 1; }
tail -1 $T/pytest.txt
timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 > $T/bench.txt 2>&1 || { tail -20 $T/bench.txt; exit 1; }
tail -1 $T/bench.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['ms_per_step'], d['breakdown_ms_per_iter'], d['roofline']['frac'])"
timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 --split --n 12500000 > $T/split.txt 2>&1 || { tail -20 $T/split.txt; exit 1; }
tail -1 $T/split.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('s12', d['ms_per_step'], d['breakdown_ms_per_iter'], d['roofline']['frac'])"
