# round-4: kernel trace of the box's FIRST GPU process (cold-start probe): where the
# first layout's extra ~15 ms goes (kernel durations vs gaps)
mkdir -p gpurun_out/t8
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/t8/trace -o run -- python3 tools/cold_start_probe.py > gpurun_out/t8/cold_trace.txt 2>&1 || { tail -20 gpurun_out/t8/cold_trace.txt; exit 1; }
grep trial gpurun_out/t8/cold_trace.txt
timeout -k 10 120 python3 tools/cold_start_probe.py > gpurun_out/t8/cold_second.txt 2>&1 || exit 1
grep trial gpurun_out/t8/cold_second.txt
