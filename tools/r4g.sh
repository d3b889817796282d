#!/bin/bash
# bench roofline with the back-to-back launch timing vs rocprof of the same command
T=gpurun_out/r4g; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --no-cpu --fit-iters 0 --steps 20 --warmup 3 > $T/bench.txt 2>&1 || { tail -20 $T/bench.txt; exit 1; }
tail -1 $T/bench.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('ms/it', round(d['ms_per_step'],4), 'frac', round(r['frac'],3), 'avg_launch_ms', round(r['avg_launch_ms'],4), 'eager', round(r['avg_launch_ms_eager_events'],4))"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/prof -o run -- python3 bench.py --no-cpu --fit-iters 0 --steps 20 --warmup 3 > $T/prof.log 2>&1 || { tail -20 $T/prof.log; exit 1; }
f=$(find $T/prof -name "*kernel_stats.csv" | head -1); cp $f $T/kernel_stats.csv
grep k_lloyd1 $T/kernel_stats.csv | cut -d, -f2-4
tail -1 $T/prof.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('under rocprof: frac', round(r['frac'],3), 'avg_launch_ms', round(r['avg_launch_ms'],4), 'eager', round(r['avg_launch_ms_eager_events'],4))"
