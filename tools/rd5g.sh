#!/bin/bash
# round 5: two-level arrival -- k_updlists phases (debug build), config-3 bench, 8-slab proxy, then the full GPU suite
T=gpurun_out/rd5g; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/lists_timing.py tools/ab/lib_dbg.so 10 100000000 1024 3 fused > $T/upd_c3.txt 2>&1 || { tail -20 $T/upd_c3.txt; exit 1; }
grep -v amdgpu.ids $T/upd_c3.txt | head -8
timeout -k 10 300 python bench.py --no-cpu --fit > $T/bench.json 2>&1 || { tail -20 $T/bench.json; exit 1; }
python3 -c "import json;d=json.loads(open('$T/bench.json').read().strip().splitlines()[-1]);print('c3', d['ms_per_step'], d['breakdown_ms_per_iter'], d['layout_ms'], d['fit'], d.get('kmeanspp_ms'))"
timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > $T/proxy8.json 2>&1 || { tail -20 $T/proxy8.json; exit 1; }
python3 -c "import json;d=json.loads(open('$T/proxy8.json').read().strip().splitlines()[-1]);print('proxy8', round(d['value'],1), d['per_rank_us'], d['centres_bitwise_equal_single_engine'])"
bash tools/prof.sh $T/prof --steps 20 --warmup 3 | tail -5 || exit 1
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $T/pytest_gpu.txt 2>&1; rc=$?
grep -E "passed|failed" $T/pytest_gpu.txt | tail -2
[ $rc -eq 0 ] || { grep -B5 -A30 "^E " $T/pytest_gpu.txt | head -60; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.txt 2>&1 || { tail -20 $T/smoke.txt; exit 1; }
tail -1 $T/smoke.txt
