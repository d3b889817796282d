#!/bin/bash
# PMC passes (tools/pmc_run.sh) of the eager bench at config 3 and at a 12.5M shard; summaries for k_lloyd and k_step.
set -o pipefail
T=gpurun_out/${1:-pmc3}; mkdir -p $T
for cfg in "c3 100000000" "s12 12500000"; do
  set -- $cfg
  bash tools/pmc_run.sh $T/$1 k_lloyd --no-graph --fit-iters 0 --steps 5 --warmup 3 --n $2 > $T/$1_k_lloyd.json || exit 1
  python tools/pmc_summary.py k_step $T/$1/*/ > $T/$1_k_step.json
done
cat $T/c3_k_lloyd.json $T/s12_k_lloyd.json
