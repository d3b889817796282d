# round-4: kernel durations of the 8-slab proxy (rocprof kernel trace): k_lloyd1, k_upd, k_lists per slab
mkdir -p gpurun_out/t14
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t14/trace -o run -- python3 bench.py --slab-of 8 --steps 20 --warmup 3 > gpurun_out/t14/p8.txt 2>&1 || { tail -5 gpurun_out/t14/p8.txt; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/t14/trace/**/*kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 2), round(float(r['MinNs'])/1e3, 2), round(float(r['MaxNs'])/1e3, 2))
PY
