#!/bin/bash
# pruning-grid size on a 12.5M shard (PCM_CELL_TARGET; >= 8 cells per centre selects the 8-slot fine-grid variant)
mkdir -p gpurun_out/cs
for t in 4096 8192 12288 16384; do
  PCM_CELL_TARGET=$t timeout -k 10 120 python bench.py --no-cpu --fit-iters 0 --split --n 12500000 > gpurun_out/cs/s12_$t.txt 2>&1 || { tail -5 gpurun_out/cs/s12_$t.txt; exit 1; }
  tail -1 gpurun_out/cs/s12_$t.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('target=$t cells', d['config']['cells'], d['config']['grid'], round(d['ms_per_step']*1e3,1), 'us/iter assign', round(d['breakdown_ms_per_iter']['assign']*1e3,1), 'cand', round(d['candidates']['mean'],2))"
done
