# round-4: cold start with Engine.reserve (first GPU process of the box), the
# reserve test, the default bench line (layout_ms/reserve_ms), a fresh-process
# probe without reserve for comparison
mkdir -p gpurun_out/t7
export PYTHONUNBUFFERED=1
PCM_RESERVE=1 timeout -k 10 120 python tools/cold_start_probe.py > gpurun_out/t7/cold_reserve.txt 2>&1 || exit 1
cat gpurun_out/t7/cold_reserve.txt
timeout -k 10 120 python tools/cold_start_probe.py > gpurun_out/t7/cold_plain.txt 2>&1 || exit 1
cat gpurun_out/t7/cold_plain.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t7/pytest.txt 2>&1 || { tail -30 gpurun_out/t7/pytest.txt; exit 1; }
tail -2 gpurun_out/t7/pytest.txt
timeout -k 10 300 python bench.py > gpurun_out/t7/bench.json 2>&1 || { tail -5 gpurun_out/t7/bench.json; exit 1; }
python3 -c "import json;b=json.loads(open('gpurun_out/t7/bench.json').read().strip().splitlines()[-1]);print(b['ms_per_step'], b['layout_ms'], b['reserve_ms'], b.get('fit'), b['roofline']['frac'])"
