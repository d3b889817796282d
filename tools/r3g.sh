#!/bin/bash
T=gpurun_out/r3g; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kpp.py tests/test_dense.py tests/test_estimator.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -40 $T/pytest.txt; exit 1; }
tail -2 $T/pytest.txt
timeout -k 10 200 python3 tools/kpp_timing.py tools/dbg/lib_dbgt.so > $T/kpp_timing.txt 2>&1 || { tail -20 $T/kpp_timing.txt; exit 1; }
cat $T/kpp_timing.txt
bash tools/kpp_prof.sh r3g/kp || exit 1
