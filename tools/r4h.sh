#!/bin/bash
# final-tree check: the driver's commands (pytest -m gpu, smoke, default bench line)
T=gpurun_out/r4h; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -60 $T/pytest.txt; exit 1; }
tail -1 $T/pytest.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.txt 2>&1 || { cat $T/smoke.txt; exit 1; }
tail -1 $T/smoke.txt
timeout -k 10 400 python bench.py > $T/bench.txt 2>&1 || { tail -20 $T/bench.txt; exit 1; }
tail -1 $T/bench.txt | cut -c1-600
