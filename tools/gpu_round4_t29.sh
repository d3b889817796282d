# round-4: the D = 4 update inside the coarse-list launch (k_updcoarse, PCM_FUSED_UPD4=1) A/B:
# parity of the D = 4 paths (both), config-5 8-way slab proxies and shard lines, kernel durations
mkdir -p gpurun_out/t29
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "d4 or random_fit or split_call" > gpurun_out/t29/pytest.txt 2>&1 || { tail -30 gpurun_out/t29/pytest.txt; exit 1; }
tail -1 gpurun_out/t29/pytest.txt
PCM_FUSED_UPD4=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_baseline_sizes.py tests/test_gpu_multirank.py tests/test_gpu_full_configs.py -x -q --timeout 700 --timeout-method thread > gpurun_out/t29/pytest_f4.txt 2>&1 || { tail -30 gpurun_out/t29/pytest_f4.txt; exit 1; }
tail -1 gpurun_out/t29/pytest_f4.txt
for V in 0 1 0 1; do
  export PCM_FUSED_UPD4=$V
  timeout -k 10 300 python bench.py --slab-of 8 --n 500000000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3 > gpurun_out/t29/c5s8_$V.json 2>&1 || { tail -5 gpurun_out/t29/c5s8_$V.json; exit 1; }
  python3 -c "import json;b=json.loads(open('gpurun_out/t29/c5s8_$V.json').read().strip().splitlines()[-1]);print('c5 slab8 fused4=$V', round(b['value'],1), 'assign', b['per_rank_us']['assign'][1:3], 'step', b['per_rank_us']['step'][1:3], b['slab_engines_agree'])"
  timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 --n 62500000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3 > gpurun_out/t29/c5_$V.json 2>&1 || { tail -5 gpurun_out/t29/c5_$V.json; exit 1; }
  python3 -c "import json;b=json.loads(open('gpurun_out/t29/c5_$V.json').read().strip().splitlines()[-1]);print('c5 shard fused4=$V', round(b['ms_per_step'],4), b['breakdown_ms_per_iter'])"
done
export PCM_FUSED_UPD4=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t29/tr -o run -- python3 bench.py --slab-of 8 --n 500000000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3 > gpurun_out/t29/tr.txt 2>&1 || { tail -5 gpurun_out/t29/tr.txt; exit 1; }
python3 - <<'PY'
import csv, glob, numpy as np
f = glob.glob('gpurun_out/t29/tr/**/*kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
for nm in ('k_lloyd1', 'k_updcoarse', 'k_upd<', 'k_coarse', 'k_lists'):
    d = np.array([(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows if nm in r['Kernel_Name']][:8 * 13])
    if len(d) > 24:
        print('c5 slab8 fused4', nm, len(d), 'after warm-up: mean %.2f p50 %.2f min %.2f max %.2f' % (d[24:].mean(), np.median(d[24:]), d[24:].min(), d[24:].max()))
PY
