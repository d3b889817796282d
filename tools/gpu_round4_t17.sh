# round-4: single-block k_upd1 (every K <= 4096) + k_lists staging with the control loads:
# GPU parity files, config-3 and config-5 lines, 8-slab proxies (c4, c5) with kernel
# durations, per-block k_lloyd1 phases of a config-5 slab (debug build)
mkdir -p gpurun_out/t17
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_compressed.py tests/test_gpu_baseline_sizes.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t17/pytest.txt 2>&1 || { tail -30 gpurun_out/t17/pytest.txt; exit 1; }
tail -1 gpurun_out/t17/pytest.txt
for W in "c3|--steps 20 --warmup 3" "c5|--n 62500000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3"; do
  tag=${W%%|*}; args=${W#*|}
  timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 $args > gpurun_out/t17/$tag.json 2>&1 || { tail -5 gpurun_out/t17/$tag.json; exit 1; }
  python3 -c "import json;b=json.loads(open('gpurun_out/t17/$tag.json').read().strip().splitlines()[-1]);print('$tag', round(b['ms_per_step'],4), b['breakdown_ms_per_iter'], round(b['roofline']['frac'],3))"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for W in "p8|--slab-of 8 --steps 20 --warmup 3" "p8c5|--slab-of 8 --n 500000000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3"; do
  tag=${W%%|*}; args=${W#*|}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t17/tr_$tag -o run -- python3 bench.py $args > gpurun_out/t17/$tag.txt 2>&1 || { tail -5 gpurun_out/t17/$tag.txt; exit 1; }
  python3 - $tag <<'PY'
import csv, glob, sys, numpy as np
tag = sys.argv[1]
f = glob.glob(f'gpurun_out/t17/tr_{tag}/**/*kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
it = 23 if tag == 'p8' else 13
for nm in ('k_lloyd1', 'k_upd', 'k_coarse', 'k_lists'):
    d = np.array([(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows if nm in r['Kernel_Name']][:8 * it])
    if len(d) > 24:
        print(tag, nm, len(d), 'slab launches after warm-up: mean %.2f p50 %.2f min %.2f max %.2f' % (d[24:].mean(), np.median(d[24:]), d[24:].min(), d[24:].max()))
PY
done
timeout -k 10 300 python tools/lloyd_timing.py $GRAFT_REPO_ROOT/tools/ab/lib_dbg.so 6 500000000 4096 4 f16 slab 8 > gpurun_out/t17/ph_c5slab.txt 2>&1 || { tail -5 gpurun_out/t17/ph_c5slab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/t17/ph_c5slab.txt
