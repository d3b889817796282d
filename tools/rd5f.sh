#!/bin/bash
# round 5: full GPU suite on the current tree + k_updlists phase timing (debug build) at config 3 and on the 8-way slab
T=gpurun_out/rd5f; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/lists_timing.py tools/ab/lib_dbg.so 10 100000000 1024 3 fused > $T/upd_c3.txt 2>&1 || { tail -20 $T/upd_c3.txt; exit 1; }
cat $T/upd_c3.txt
timeout -k 10 300 python tools/lists_timing.py tools/ab/lib_dbg.so 10 100000000 1024 3 fused slab 8 > $T/upd_s8.txt 2>&1 || { tail -20 $T/upd_s8.txt; exit 1; }
cat $T/upd_s8.txt
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $T/pytest_gpu.txt 2>&1; rc=$?
grep -E "passed|failed" $T/pytest_gpu.txt | tail -2
[ $rc -eq 0 ] || { grep -B5 -A30 "^E " $T/pytest_gpu.txt | head -60; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.txt 2>&1 || { tail -20 $T/smoke.txt; exit 1; }
tail -1 $T/smoke.txt
