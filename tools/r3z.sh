#!/bin/bash
# labels back to row order through the sort's position maps: full GPU suite, bench fit, rocprof of the fit kernels
T=gpurun_out/r3z; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -60 $T/pytest.txt; exit 1; }
tail -1 $T/pytest.txt
for M in 3 1; do
  PCM_UNPERM=$M timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 3 > $T/bench$M.txt 2>&1 || { tail -20 $T/bench$M.txt; exit 1; }
  tail -1 $T/bench$M.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('unperm=$M ms/it', round(d['ms_per_step'],4), 'layout', d.get('layout_ms'), 'fit', d.get('fit'))"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/prof -o run -- python3 bench.py --no-cpu --steps 10 --warmup 3 > $T/prof.log 2>&1 || { tail -20 $T/prof.log; exit 1; }
f=$(find $T/prof -name "*kernel_stats.csv" | head -1); cp $f $T/kernel_stats.csv
grep -E "k_lab_gather|k_label|k_rs_scatter|k_unpermute|k_tile_compress|k_bbox_partial" $T/kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
