#!/bin/bash
# A/B of an environment switch on the config-5 shard (62.5M, K=4096, D=4) and the 8-way slab proxy, alternating:
#   tools/ab_c5.sh OUT VAR "v1 v2" REPS
set -o pipefail
T=gpurun_out/$1; VAR=$2; VALS=$3; REPS=$4; mkdir -p $T
for r in $(seq $REPS); do for v in $VALS; do
  env $VAR=$v timeout -k 10 200 python bench.py --no-cpu --no-kpp --fit-iters 0 --n 62500000 --k 4096 --d 4 > $T/c5_${v}_$r.json 2> $T/err.txt || { tail -20 $T/err.txt; exit 1; }
  tail -1 $T/c5_${v}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown_ms_per_iter']; print('c5 shard $VAR=$v', 'us/iter', round(d['ms_per_step']*1e3,1), 'assign', round(b['assign']*1e3,1), 'frac', d['roofline']['frac'])"
  env $VAR=$v timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > $T/s8_${v}_$r.json 2> $T/err.txt || { tail -20 $T/err.txt; exit 1; }
  tail -1 $T/s8_${v}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('slab8 $VAR=$v', 'us/rank', round(d['value'],1), 'assign', d['per_rank_us']['assign'], 'bitwise', d['centres_bitwise_equal_single_engine'])"
done; done
