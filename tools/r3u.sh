#!/bin/bash
# spread same-address atomics (k_step arrival, k_label inertia, k_tile_compress counter): full GPU suite, bench, rocprof, slab proxy 8
T=gpurun_out/r3u; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -60 $T/pytest.txt; exit 1; }
tail -1 $T/pytest.txt
timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 3 > $T/bench.txt 2>&1 || { tail -20 $T/bench.txt; exit 1; }
tail -1 $T/bench.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/it', round(d['ms_per_step'],4), 'brk', d.get('breakdown_ms_per_iter'), 'layout', d.get('layout_ms'), 'fit', d.get('fit'))"
timeout -k 10 300 python bench.py --slab-of 8 --steps 20 --warmup 3 > $T/proxy8.json 2>&1 || { tail -20 $T/proxy8.json; exit 1; }
tail -1 $T/proxy8.json | cut -c1-420
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/prof -o run -- python3 bench.py --no-cpu --steps 20 --warmup 3 > $T/prof.log 2>&1 || { tail -20 $T/prof.log; exit 1; }
f=$(find $T/prof -name "*kernel_stats.csv" | head -1); cp $f $T/kernel_stats.csv
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open("gpurun_out/r3u/kernel_stats.csv")))[:16]:
    n=r["Name"]; n=n.split("(")[0][-60:] if "rocprim" not in n else "rocprim:"+n.split("detail::")[-1][:50]
    print(f"{n:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us")
PY
