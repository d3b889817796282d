# round-4: cold start after moving the statistics tensor (torch's first kernel) to
# engine creation -- the box's FIRST GPU process is the bench's default line --, then
# the probe, the GPU suite and smoke
mkdir -p gpurun_out/t9
export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py > gpurun_out/t9/bench_first.json 2>&1 || { tail -5 gpurun_out/t9/bench_first.json; exit 1; }
python3 -c "import json;b=json.loads(open('gpurun_out/t9/bench_first.json').read().strip().splitlines()[-1]);print('first-process bench: ms/step', b['ms_per_step'], 'layout_ms', b['layout_ms'], 'reserve_ms', b['reserve_ms'], b.get('fit'), 'frac', b['roofline']['frac'])"
timeout -k 10 120 python tools/cold_start_probe.py > gpurun_out/t9/cold.txt 2>&1 || exit 1
grep trial gpurun_out/t9/cold.txt
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t9/pytest.txt 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/t9/pytest.txt | tail -5
[ $rc -eq 0 ] || { grep -B5 -A30 "^E " gpurun_out/t9/pytest.txt | head -60; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t9/smoke.txt 2>&1 || { tail -20 gpurun_out/t9/smoke.txt; exit 1; }
tail -3 gpurun_out/t9/smoke.txt
