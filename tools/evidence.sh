#!/bin/bash
# Round evidence on the GPU box: GPU tests, smoke, headline bench (with CPU baseline
# and a 20-iteration fit), rocprofv3 kernel stats, HBM traffic PMC passes.
# usage: tools/evidence.sh TAG   -> gpurun_out/ev_TAG/
T=gpurun_out/ev_$1; mkdir -p $T
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $T/pytest_gpu.txt 2>&1 || { tail -30 $T/pytest_gpu.txt; exit 1; }
tail -2 $T/pytest_gpu.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.txt 2>&1 || { cat $T/smoke.txt; exit 1; }
tail -1 $T/smoke.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $T/pmc_$P -o run -- python3 bench.py --no-cpu --no-graph --fit-iters 0 --steps 5 --warmup 3 > $T/pmc_$P.log 2>&1 || { echo "FAIL pmc $P"; tail -5 $T/pmc_$P.log; exit 1; }
done
python tools/pmc_summary.py k_lloyd $T/pmc_FETCH_SIZE $T/pmc_WRITE_SIZE > $T/pmc_k_lloyd.json && cat $T/pmc_k_lloyd.json
bash tools/prof.sh $T/prof --steps 20 --warmup 3 --fit | tail -14 || exit 1
PCM_PMC_JSON=$T/pmc_k_lloyd.json timeout -k 10 400 python bench.py --fit --cloud --stereo > $T/bench.txt 2>&1 || { tail -20 $T/bench.txt; exit 1; }
tail -1 $T/bench.txt
timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 --n 62500000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3 > $T/c5.txt 2>&1 || { tail -20 $T/c5.txt; exit 1; }
tail -1 $T/c5.txt | cut -c1-300
timeout -k 10 300 python bench.py --slab-of 8 --n 500000000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3 > $T/proxy8_c5.json 2>&1 || { tail -20 $T/proxy8_c5.json; exit 1; }
tail -1 $T/proxy8_c5.json | cut -c1-400
for P in 2 4 8; do
  timeout -k 10 200 python bench.py --slab-of $P --steps 20 --warmup 3 > $T/proxy$P.json 2>&1 || { tail -20 $T/proxy$P.json; exit 1; }
  tail -1 $T/proxy$P.json | cut -c1-400
done
timeout -k 10 200 python bench.py --gpus 2 --backend gloo --n 20000000 --no-cpu --fit-iters 0 --steps 5 --warmup 2 > $T/gloo2.txt 2>&1 || { tail -20 $T/gloo2.txt; exit 1; }
tail -1 $T/gloo2.txt | cut -c1-300
