# round-4: single-block k_upd1 (K <= 4096), k_lists staging with the control loads, and the
# fused k_updlists (PCM_FUSED_UPD=1, D <= 3, K <= 1024) A/B, the z-at-top record decode A/B: GPU parity files (both paths),
# config-3 / config-5 lines, 8-slab proxies with kernel durations, config-5 slab k_lloyd1 phases
mkdir -p gpurun_out/t18
export PYTHONUNBUFFERED=1
T="tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_compressed.py tests/test_gpu_baseline_sizes.py"
timeout -k 10 700 python -u -m pytest $T -x -q --timeout 200 --timeout-method thread > gpurun_out/t18/pytest.txt 2>&1 || { tail -30 gpurun_out/t18/pytest.txt; exit 1; }
tail -1 gpurun_out/t18/pytest.txt
PCM_FUSED_UPD=1 timeout -k 10 700 python -u -m pytest $T tests/test_gpu_crowded.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t18/pytest_fused.txt 2>&1 || { tail -30 gpurun_out/t18/pytest_fused.txt; exit 1; }
tail -1 gpurun_out/t18/pytest_fused.txt
for V in split fused; do
  if [ $V = fused ]; then export PCM_FUSED_UPD=1; else unset PCM_FUSED_UPD; fi
  timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 --steps 20 --warmup 3 > gpurun_out/t18/c3_$V.json 2>&1 || { tail -5 gpurun_out/t18/c3_$V.json; exit 1; }
  python3 -c "import json;b=json.loads(open('gpurun_out/t18/c3_$V.json').read().strip().splitlines()[-1]);print('c3 $V', round(b['ms_per_step'],4), b['breakdown_ms_per_iter'], round(b['roofline']['frac'],3))"
  timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > gpurun_out/t18/p8_$V.json 2>&1 || { tail -5 gpurun_out/t18/p8_$V.json; exit 1; }
  python3 -c "import json;b=json.loads(open('gpurun_out/t18/p8_$V.json').read().strip().splitlines()[-1]);print('p8 $V', round(b['value'],2), b['per_rank_us'], b['centres_bitwise_equal_single_engine'])"
done
unset PCM_FUSED_UPD
for V in zt0 ztop zt0 ztop; do   # compressed-record decode: z field at the top (build) vs after y
  if [ $V = zt0 ]; then export PCM_SO=$GRAFT_REPO_ROOT/tools/ab/lib_zt0.so; else unset PCM_SO; fi
  timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 --steps 20 --warmup 3 > gpurun_out/t18/c3_$V.json 2>&1 || { tail -5 gpurun_out/t18/c3_$V.json; exit 1; }
  python3 -c "import json;b=json.loads(open('gpurun_out/t18/c3_$V.json').read().strip().splitlines()[-1]);print('c3 $V', round(b['ms_per_step'],4), round(b['roofline']['avg_launch_ms'],4), round(b['roofline']['avg_launch_ms_back_to_back'],4))"
done
unset PCM_SO
timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 --n 62500000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3 > gpurun_out/t18/c5.json 2>&1 || { tail -5 gpurun_out/t18/c5.json; exit 1; }
python3 -c "import json;b=json.loads(open('gpurun_out/t18/c5.json').read().strip().splitlines()[-1]);print('c5', round(b['ms_per_step'],4), b['breakdown_ms_per_iter'], round(b['roofline']['frac'],3))"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for W in "p8|--slab-of 8 --steps 20 --warmup 3|" "p8f|--slab-of 8 --steps 20 --warmup 3|1" "p8c5|--slab-of 8 --n 500000000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3|"; do
  tag=$(echo "$W" | cut -d'|' -f1); args=$(echo "$W" | cut -d'|' -f2); fz=$(echo "$W" | cut -d'|' -f3)
  if [ -n "$fz" ]; then export PCM_FUSED_UPD=1; else unset PCM_FUSED_UPD; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t18/tr_$tag -o run -- python3 bench.py $args > gpurun_out/t18/$tag.txt 2>&1 || { tail -5 gpurun_out/t18/$tag.txt; exit 1; }
  python3 - $tag <<'PY'
import csv, glob, sys, numpy as np
tag = sys.argv[1]
f = glob.glob(f'gpurun_out/t18/tr_{tag}/**/*kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
it = 13 if tag == 'p8c5' else 23
for nm in ('k_lloyd1', 'k_upd', 'k_coarse', 'k_lists'):
    d = np.array([(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows if nm in r['Kernel_Name']][:8 * it])
    if len(d) > 24:
        print(tag, nm, len(d), 'slab launches after warm-up: mean %.2f p50 %.2f min %.2f max %.2f' % (d[24:].mean(), np.median(d[24:]), d[24:].min(), d[24:].max()))
PY
done
unset PCM_FUSED_UPD
timeout -k 10 300 python tools/lloyd_timing.py $GRAFT_REPO_ROOT/tools/ab/lib_dbg.so 6 500000000 4096 4 f16 slab 8 > gpurun_out/t18/ph_c5slab.txt 2>&1 || { tail -5 gpurun_out/t18/ph_c5slab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/t18/ph_c5slab.txt
