#!/bin/bash
# k-means++ dense-step row pass in apply: parity, per-step means
T=gpurun_out/r4b; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kpp.py tests/test_dense.py tests/test_estimator.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -60 $T/pytest.txt; exit 1; }
tail -1 $T/pytest.txt
timeout -k 10 300 bash tools/kpp_prof.sh r4b_prof > $T/kpp_prof.txt 2>&1 || { tail -20 $T/kpp_prof.txt; exit 1; }
tail -5 $T/kpp_prof.txt
