#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/p
timeout -k 10 120 python tools/step_timing2.py $PWD/tools/variants/lib_dbgt.so 10 62500000 4096 4 > gpurun_out/p/st_c5.txt 2>&1 || { tail -5 gpurun_out/p/st_c5.txt; exit 1; }
cat gpurun_out/p/st_c5.txt | grep -v amdgpu.ids
timeout -k 10 120 python tools/step_timing2.py $PWD/tools/variants/lib_dbgt.so 10 12500000 1024 3 > gpurun_out/p/st_s12.txt 2>&1 || { tail -5 gpurun_out/p/st_s12.txt; exit 1; }
cat gpurun_out/p/st_s12.txt | grep -v amdgpu.ids
