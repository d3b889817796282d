# round-4: LSD record sort with 512-thread chunks of 8192 items (tools/ab/lib_rs512.so, -DPCM_RS_TPB=512)
# vs the build's 256 x 16 = 4096: parity with the variant, then alternating layout / fit timings
mkdir -p gpurun_out/t24
export PYTHONUNBUFFERED=1
PCM_SO=$GRAFT_REPO_ROOT/tools/ab/lib_rs512.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compressed.py tests/test_gpu_baseline_sizes.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t24/pytest.txt 2>&1 || { tail -30 gpurun_out/t24/pytest.txt; exit 1; }
tail -1 gpurun_out/t24/pytest.txt
for V in b256 rs512 b256 rs512; do
  if [ $V = rs512 ]; then export PCM_SO=$GRAFT_REPO_ROOT/tools/ab/lib_rs512.so; else unset PCM_SO; fi
  timeout -k 10 200 python bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/t24/c3_$V.json 2>&1 || { tail -5 gpurun_out/t24/c3_$V.json; exit 1; }
  python3 -c "import json;b=json.loads(open('gpurun_out/t24/c3_$V.json').read().strip().splitlines()[-1]);print('$V layout_ms', round(b['layout_ms'],3), 'fit', b['fit'])"
done
unset PCM_SO
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PCM_SO=$GRAFT_REPO_ROOT/tools/ab/lib_rs512.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t24/tr -o run -- python3 bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/t24/tr.txt 2>&1 || { tail -5 gpurun_out/t24/tr.txt; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/t24/tr/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'k_rs_' in r['Name']:
        print('rs512', r['Name'][:48], r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
PY
