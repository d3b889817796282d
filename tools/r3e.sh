#!/bin/bash
# round 3: LDS counting-sort layout -- layout-sensitive GPU parity, A/B vs radix, rocprof of the layout kernels
T=gpurun_out/r3e; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py tests/test_gpu_multirank.py tests/test_kpp.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -40 $T/pytest.txt; exit 1; }
tail -2 $T/pytest.txt
for L in 0 1; do
  PCM_LAYOUT_RADIX=$L timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 3 > $T/bench_radix$L.txt 2>&1 || { tail -20 $T/bench_radix$L.txt; exit 1; }
  tail -1 $T/bench_radix$L.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('radix=$L', 'layout_ms', round(d['layout_ms'],2), 'fit', d['fit'], 'ms/it', round(d['ms_per_step'],4))"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/prof -o run -- python3 bench.py --no-cpu --steps 20 --warmup 3 > $T/prof.txt 2>&1 || { tail -20 $T/prof.txt; exit 1; }
f=$(find $T/prof -name "*kernel_stats.csv" | head -1); cp "$f" $T/kernel_stats.csv
python3 - "$T/kernel_stats.csv" <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:16]:
    print(f'{r["Name"][:60]:60s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:9.2f} min_us={float(r["MinNs"])/1e3:9.2f}')
PY
echo "== kpp search phase stamps (debug build)"
timeout -k 10 200 python3 tools/kpp_timing.py tools/dbg/lib_dbgt.so > $T/kpp_timing.txt 2>&1 || { tail -20 $T/kpp_timing.txt; exit 1; }
cat $T/kpp_timing.txt
echo "== kpp per-step kernel trace (batched cells)"
bash tools/kpp_prof.sh r3e/kp || exit 1
