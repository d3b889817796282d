#!/bin/bash
# k-means++ without same-address atomic storms: parity, timing, per-step kernel means, phase stamps
T=gpurun_out/r3t; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kpp.py tests/test_dense.py tests/test_estimator.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -60 $T/pytest.txt; exit 1; }
tail -1 $T/pytest.txt
timeout -k 10 300 python tools/kpp_bench.py 100000000 1024 3 > $T/kpp.txt 2>&1 || { tail -20 $T/kpp.txt; exit 1; }
grep -v amdgpu $T/kpp.txt
timeout -k 10 300 bash tools/kpp_prof.sh r3t_prof > $T/kpp_prof.txt 2>&1 || { tail -20 $T/kpp_prof.txt; exit 1; }
tail -5 $T/kpp_prof.txt
timeout -k 10 300 python tools/kpp_timing.py tools/variants/lib_dbg.so > $T/kpp_timing.txt 2>&1 || { tail -20 $T/kpp_timing.txt; exit 1; }
grep -v amdgpu.ids $T/kpp_timing.txt
