#!/bin/bash
set -o pipefail
T=gpurun_out/${1:-st}; mkdir -p $T
L=$PWD/tools/variants/lib_dbgt.so
for cfg in "s12 12500000 1024 3 0" "c3 100000000 1024 3 0" "c3b2 100000000 1024 3 2"; do
  set -- $cfg
  if [ $5 = 0 ]; then unset PCM_CAND_BPC_RT; else export PCM_CAND_BPC_RT=$5; fi
  timeout -k 10 120 python tools/step_timing2.py $L 10 $2 $3 $4 > $T/st_$1.txt 2>&1 || { tail -5 $T/st_$1.txt; exit 1; }
  grep -v amdgpu.ids $T/st_$1.txt | grep -v "block start\|slowest"
done
unset PCM_CAND_BPC_RT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -30 $T/pytest.txt; exit 1; }
tail -1 $T/pytest.txt
for b in 0 2; do
  if [ $b = 0 ]; then unset PCM_CAND_BPC_RT; else export PCM_CAND_BPC_RT=$b; fi
  timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 > $T/bench$b.txt 2>&1 || { tail -20 $T/bench$b.txt; exit 1; }
  tail -1 $T/bench$b.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 bpc$b', d['ms_per_step'], d['breakdown_ms_per_iter'], d['roofline']['frac'])"
done
unset PCM_CAND_BPC_RT
timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 --split --n 12500000 > $T/split.txt 2>&1 || { tail -20 $T/split.txt; exit 1; }
tail -1 $T/split.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('s12', d['ms_per_step'], d['breakdown_ms_per_iter'], d['roofline']['frac'])"
