# round-4: final tree -- the GPU suite and smoke
mkdir -p gpurun_out/t30
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t30/pytest.txt 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/t30/pytest.txt | tail -2
[ $rc -eq 0 ] || { grep -B5 -A30 "^E " gpurun_out/t30/pytest.txt | head -60; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t30/smoke.txt 2>&1 || { tail -20 gpurun_out/t30/smoke.txt; exit 1; }
tail -1 gpurun_out/t30/smoke.txt
timeout -k 10 300 python bench.py > gpurun_out/t30/bench.json 2>&1 || { tail -5 gpurun_out/t30/bench.json; exit 1; }
python3 -c "import json;b=json.loads(open('gpurun_out/t30/bench.json').read().strip().splitlines()[-1]);print('bench', b['value'], b['ms_per_step'], b['layout_ms'], b.get('fit'), round(b['roofline']['frac'],3))"
