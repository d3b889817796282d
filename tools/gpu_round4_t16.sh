# round-4: k_upd1 with every load in one latency: parity files, 8-slab proxy kernel durations
mkdir -p gpurun_out/t16
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_compressed.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t16/pytest.txt 2>&1 || { tail -30 gpurun_out/t16/pytest.txt; exit 1; }
tail -1 gpurun_out/t16/pytest.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t16/trace -o run -- python3 bench.py --slab-of 8 --steps 20 --warmup 3 > gpurun_out/t16/p8.txt 2>&1 || { tail -5 gpurun_out/t16/p8.txt; exit 1; }
python3 - <<'PY'
import csv, glob, numpy as np
f = glob.glob('gpurun_out/t16/trace/**/*kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
for nm in ('k_lloyd1', 'k_upd', 'k_lists'):
    d = np.array([(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows if nm in r['Kernel_Name']][:184])
    print(nm, len(d), 'slab launches after warm-up: mean %.2f p50 %.2f min %.2f max %.2f' % (d[24:].mean(), np.median(d[24:]), d[24:].min(), d[24:].max()))
PY
