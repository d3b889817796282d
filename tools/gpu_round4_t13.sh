# round-4: per-block phase times of k_lloyd1 (debug build, tools/lloyd_timing.py) at
# config 3 and at a 12.5M-point cloud (one slab's size)
mkdir -p gpurun_out/t13
export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/lloyd_timing.py $GRAFT_REPO_ROOT/tools/ab/lib_dbg.so 10 > gpurun_out/t13/c3.txt 2>&1 || { tail -5 gpurun_out/t13/c3.txt; exit 1; }
cat gpurun_out/t13/c3.txt | grep -v amdgpu.ids
timeout -k 10 200 python tools/lloyd_timing.py $GRAFT_REPO_ROOT/tools/ab/lib_dbg.so 10 12500000 1024 3 > gpurun_out/t13/s12.txt 2>&1 || { tail -5 gpurun_out/t13/s12.txt; exit 1; }
cat gpurun_out/t13/s12.txt | grep -v amdgpu.ids
