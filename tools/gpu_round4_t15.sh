# round-4: single-block k_upd1 (K <= 2048): GPU suite, config-3 line, 8-slab proxy + its kernel durations
mkdir -p gpurun_out/t15
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t15/pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/t15/pytest.txt
[ $rc -eq 0 ] || { grep -B5 -A30 "^E " gpurun_out/t15/pytest.txt | head -60; exit $rc; }
timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 --steps 20 --warmup 3 > gpurun_out/t15/c3.json 2>&1 || { tail -5 gpurun_out/t15/c3.json; exit 1; }
python3 -c "import json;b=json.loads(open('gpurun_out/t15/c3.json').read().strip().splitlines()[-1]);print('c3', round(b['ms_per_step'],4), b['breakdown_ms_per_iter'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t15/trace -o run -- python3 bench.py --slab-of 8 --steps 20 --warmup 3 > gpurun_out/t15/p8.txt 2>&1 || { tail -5 gpurun_out/t15/p8.txt; exit 1; }
tail -1 gpurun_out/t15/p8.txt | cut -c1-400
python3 - <<'PY'
import csv, glob, numpy as np
f = glob.glob('gpurun_out/t15/trace/**/*kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
for nm in ('k_lloyd1', 'k_upd', 'k_lists'):
    d = np.array([(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows if nm in r['Kernel_Name']][:184])
    print(nm, len(d), 'slab launches after warm-up: mean %.2f p50 %.2f min %.2f max %.2f' % (d[24:].mean(), np.median(d[24:]), d[24:].min(), d[24:].max()))
PY
