# round-4: D <= 3 list blocks of 256 threads (PCM_LISTS3_TPB=256) and 2 blocks per coarse cell
# (PCM_CAND_BPC_RT=2) on the split update path (PCM_FUSED_UPD=0), config 3 and the 8-way slab
mkdir -p gpurun_out/t28
export PYTHONUNBUFFERED=1 PCM_FUSED_UPD=0
PCM_LISTS3_TPB=256 PCM_CAND_BPC_RT=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t28/pytest.txt 2>&1 || { tail -30 gpurun_out/t28/pytest.txt; exit 1; }
tail -1 gpurun_out/t28/pytest.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for V in "512|1|" "256|1|256" "256|2|256" "512|2|"; do
  tpb=$(echo "$V" | cut -d'|' -f1); bpc=$(echo "$V" | cut -d'|' -f2); lt=$(echo "$V" | cut -d'|' -f3)
  if [ -n "$lt" ]; then export PCM_LISTS3_TPB=$lt; else unset PCM_LISTS3_TPB; fi
  export PCM_CAND_BPC_RT=$bpc
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t28/tr_${tpb}_$bpc -o run -- python3 bench.py --no-cpu --fit-iters 0 --steps 10 --warmup 3 > gpurun_out/t28/c3_${tpb}_$bpc.txt 2>&1 || { tail -5 gpurun_out/t28/c3_${tpb}_$bpc.txt; exit 1; }
  python3 - ${tpb}_$bpc <<'PY'
import csv, glob, sys
tag = sys.argv[1]
f = glob.glob(f'gpurun_out/t28/tr_{tag}/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r['Name'] for k in ('k_lists', 'k_upd1', 'k_lloyd1')):
        print('c3 tpb_bpc', tag, r['Name'][:40], r['Calls'], round(float(r['AverageNs']) / 1e3, 2))
PY
done
