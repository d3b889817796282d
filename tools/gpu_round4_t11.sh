# round-4: wave-contiguous compressed stream (PCM_ZWAVE=1, the build) vs the
# per-lane 32-B records (tools/ab/lib_zw0.so): parity, then alternating c3 lines
mkdir -p gpurun_out/t11
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compressed.py tests/test_gpu_crowded.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t11/pytest.txt 2>&1 || { tail -30 gpurun_out/t11/pytest.txt; exit 1; }
tail -1 gpurun_out/t11/pytest.txt
for i in 1 2; do
  for V in new old; do
    if [ $V = old ]; then export PCM_SO=$GRAFT_REPO_ROOT/tools/ab/lib_zw0.so; else unset PCM_SO; fi
    timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 --steps 20 --warmup 3 > gpurun_out/t11/c3_$V$i.json 2>&1 || { tail -5 gpurun_out/t11/c3_$V$i.json; exit 1; }
    python3 -c "import json;b=json.loads(open('gpurun_out/t11/c3_$V$i.json').read().strip().splitlines()[-1]);print('$V$i', round(b['ms_per_step'],4), round(b['roofline']['avg_launch_ms'],4), round(b['roofline']['avg_launch_ms_back_to_back'],4))"
  done
done
unset PCM_SO
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t11/trace -o run -- python3 bench.py --no-cpu --fit-iters 0 --steps 20 --warmup 3 > gpurun_out/t11/trace.txt 2>&1 || { tail -5 gpurun_out/t11/trace.txt; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/t11/trace/**/*kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:3]:
    print(r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3, float(r['MaxNs'])/1e3)
PY
timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/t11/pmc1 -o run -- python3 bench.py --no-cpu --fit-iters 0 --no-graph --steps 5 --warmup 3 > gpurun_out/t11/pmc1.log 2>&1 || exit 1
python3 tools/pmc_summary.py k_lloyd1 gpurun_out/t11/pmc1 | grep -E "FETCH|_ns|hbm"
