# round-4: GPU test suite, then the measurements of gpu_round4_t2.sh
mkdir -p gpurun_out/t3
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t3/pytest.txt 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/t3/pytest.txt | tail -5
[ $rc -eq 0 ] || { grep -B5 -A30 "^E " gpurun_out/t3/pytest.txt | head -60; exit $rc; }
bash tools/gpu_round4_t2.sh
