# round-4: label gathers with 4 outputs per thread (k_lab_gather4): parity of everything that
# uses labels, the whole-fit line, and k_label's rocprof average
mkdir -p gpurun_out/t27
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compressed.py tests/test_gpu_baseline_sizes.py tests/test_gpu_crowded.py tests/test_gpu_multirank.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t27/pytest.txt 2>&1 || { tail -30 gpurun_out/t27/pytest.txt; exit 1; }
tail -1 gpurun_out/t27/pytest.txt
timeout -k 10 200 python bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/t27/c3.json 2>&1 || { tail -5 gpurun_out/t27/c3.json; exit 1; }
python3 -c "import json;b=json.loads(open('gpurun_out/t27/c3.json').read().strip().splitlines()[-1]);print('layout_ms', round(b['layout_ms'],3), 'fit', b['fit'], 'ms/step', b['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t27/tr -o run -- python3 bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/t27/tr.txt 2>&1 || { tail -5 gpurun_out/t27/tr.txt; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/t27/tr/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r['Name'] for k in ('k_label', 'k_lab_gather4', 'k_lloyd1', 'k_updlists')):
        print(r['Name'][:48], r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
PY
