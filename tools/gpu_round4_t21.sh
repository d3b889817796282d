# round-4: per-block phase times of the list update (debug build, tools/lists_timing.py):
# config-5 8-way slab (k_lists<4,2>), config-4 8-way slab and config 3 (k_lists<3,4,STAGE>)
mkdir -p gpurun_out/t21
export PYTHONUNBUFFERED=1
L=$GRAFT_REPO_ROOT/tools/ab/lib_dbg.so
timeout -k 10 300 python tools/lists_timing.py $L 6 500000000 4096 4 f16 slab 8 > gpurun_out/t21/c5slab.txt 2>&1 || { tail -5 gpurun_out/t21/c5slab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/t21/c5slab.txt
timeout -k 10 200 python tools/lists_timing.py $L 6 100000000 1024 3 slab 8 > gpurun_out/t21/c4slab.txt 2>&1 || { tail -5 gpurun_out/t21/c4slab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/t21/c4slab.txt
timeout -k 10 200 python tools/lists_timing.py $L 6 100000000 1024 3 > gpurun_out/t21/c3.txt 2>&1 || { tail -5 gpurun_out/t21/c3.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/t21/c3.txt
