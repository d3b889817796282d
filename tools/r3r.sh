#!/bin/bash
# k-means++ phase stamps (debug build): last search and eval launches at config 3
T=gpurun_out/r3r; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/kpp_timing.py tools/variants/lib_dbg.so > $T/kpp_timing.txt 2>&1 || { tail -20 $T/kpp_timing.txt; exit 1; }
grep -v amdgpu.ids $T/kpp_timing.txt
