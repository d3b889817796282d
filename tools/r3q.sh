#!/bin/bash
# layout A/B: record sort (default) vs (key,row) pairs + row gather; parity subset; rocprof of the record sort
T=gpurun_out/r3q; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compressed.py tests/test_gpu_crowded.py tests/test_gpu_baseline_sizes.py tests/test_kpp.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -60 $T/pytest.txt; exit 1; }
tail -2 $T/pytest.txt
for V in prod; do
  SO=""; [ $V = ipt8 ] && SO=tools/variants/lib_ipt8.so
  PCM_SO=$SO timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 3 > $T/bench_$V.txt 2>&1 || { tail -20 $T/bench_$V.txt; exit 1; }
  tail -1 $T/bench_$V.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$V ms/it', round(d['ms_per_step'],4), 'layout', d.get('layout_ms'), 'fit', d.get('fit'))"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/prof -o run -- python3 bench.py --no-cpu --steps 5 --warmup 3 > $T/prof.log 2>&1 || { tail -20 $T/prof.log; exit 1; }
f=$(find $T/prof -name "*kernel_stats.csv" | head -1); cp $f $T/kernel_stats.csv
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/r3q/kernel_stats.csv")):
    n=r["Name"]; n=n.split("(")[0][-60:] if "rocprim" not in n else "rocprim:"+n.split("detail::")[-1][:50]
    print(f"{n:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us")
PY
timeout -k 10 300 python tools/kpp_bench.py 100000000 1024 3 > $T/kpp.txt 2>&1 || { tail -20 $T/kpp.txt; exit 1; }
tail -4 $T/kpp.txt
timeout -k 10 300 python tools/kpp_counts.py tools/variants/lib_dbg.so > $T/kpp_counts.txt 2>&1 || { tail -20 $T/kpp_counts.txt; exit 1; }
cat $T/kpp_counts.txt | grep -v amdgpu.ids
