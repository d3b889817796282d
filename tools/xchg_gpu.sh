#!/bin/bash
# peer exchange on one GPU: exchange tests, multi-process tests, 8-slab proxy with and without it
# usage: tools/xchg_gpu.sh OUT [quick]   (quick: skip the multi-process tests)
set -o pipefail
T=gpurun_out/${1:-xg}; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_xchg.py -m gpu -x -v --timeout 120 --timeout-method thread > $T/pytest_xchg.txt 2>&1 || { tail -40 $T/pytest_xchg.txt; exit 1; }
tail -1 $T/pytest_xchg.txt
if [ "$2" != quick ]; then
timeout -k 10 500 python -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v --timeout 150 --timeout-method thread > $T/pytest_multirank.txt 2>&1 || { tail -40 $T/pytest_multirank.txt; exit 1; }
tail -1 $T/pytest_multirank.txt
fi
run() {  # name, env..., args
  name=$1; shift
  e=(); while [ "$1" != -- ]; do e+=("$1"); shift; done; shift
  env "${e[@]}" timeout -k 10 200 python bench.py --slab-of 8 --steps 40 --warmup 5 --no-cpu "$@" > $T/proxy8_$name.json 2> $T/proxy8_$name.err || { tail -20 $T/proxy8_$name.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$T/proxy8_$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value'],2), d['per_rank_us'], d['centres_bitwise_equal_single_engine'])"
}
run peer PCM_XCHG_WT=1 -- --exchange peer
run peer_fenced PCM_XCHG_WT=0 -- --exchange peer
run collective PCM_XCHG_WT=1 -- --exchange collective
run peer2 PCM_XCHG_WT=1 -- --exchange peer
