#!/bin/bash
# Round evidence on the GPU box: GPU tests, smoke, HBM traffic PMC passes, rocprofv3 kernel stats,
# the headline bench line (CPU baselines, whole fit, k-means++, cloud and stereo legs), the config-2
# line, the config-5 shard, the 8-slab proxies (configs 4 and 5), the multi-GPU call sequence
# (RCCL group of 1) replayed from a graph and launched eagerly, and a 2-rank gloo rehearsal; round 6:
# the slab proxies with the peer exchange (and host-summed), a kernel trace of the 8-slab proxy, and the
# config-5 shard's counter set (tools/kernel_profile.sh).
# usage: tools/evidence.sh TAG [skip-tests]   -> gpurun_out/ev_TAG/
T=gpurun_out/ev_$1; mkdir -p $T
export PYTHONUNBUFFERED=1
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=25 > $T/pytest_gpu.txt 2>&1 || { grep -B5 -A30 "^E " $T/pytest_gpu.txt | head -60; exit 1; }
  grep -E "passed|failed" $T/pytest_gpu.txt | tail -1
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.txt 2>&1 || { cat $T/smoke.txt; exit 1; }
  tail -1 $T/smoke.txt
fi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $T/pmc_$P -o run -- python3 bench.py --no-cpu --no-graph --fit-iters 0 --steps 5 --warmup 3 > $T/pmc_$P.log 2>&1 || { echo "FAIL pmc $P"; tail -5 $T/pmc_$P.log; exit 1; }
done
python tools/pmc_summary.py k_lloyd $T/pmc_FETCH_SIZE $T/pmc_WRITE_SIZE > $T/pmc_k_lloyd.json && cat $T/pmc_k_lloyd.json
bash tools/prof.sh $T/prof --steps 20 --warmup 3 --fit | tail -14 || exit 1
PCM_PMC_JSON=$T/pmc_k_lloyd.json timeout -k 10 400 python bench.py --fit --cloud --stereo > $T/bench.txt 2>&1 || { tail -20 $T/bench.txt; exit 1; }
tail -1 $T/bench.txt | cut -c1-400
timeout -k 10 300 python bench.py --config 2 --fit-iters 20 > $T/c2.txt 2>&1 || { tail -20 $T/c2.txt; exit 1; }
tail -1 $T/c2.txt | cut -c1-300
timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 --n 62500000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3 > $T/c5.txt 2>&1 || { tail -20 $T/c5.txt; exit 1; }
tail -1 $T/c5.txt | cut -c1-300
timeout -k 10 300 python bench.py --slab-of 8 --n 500000000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3 > $T/proxy8_c5.json 2>&1 || { tail -20 $T/proxy8_c5.json; exit 1; }
tail -1 $T/proxy8_c5.json | cut -c1-400
for P in 2 4 8; do
  timeout -k 10 200 python bench.py --slab-of $P --steps 20 --warmup 3 > $T/proxy$P.json 2>&1 || { tail -20 $T/proxy$P.json; exit 1; }
  tail -1 $T/proxy$P.json | cut -c1-300
done
timeout -k 10 200 python bench.py --slab-of 8 --exchange collective --steps 20 --warmup 3 > $T/proxy8_collective.json 2>&1 || { tail -20 $T/proxy8_collective.json; exit 1; }
tail -1 $T/proxy8_collective.json | cut -c1-300
bash tools/prof_proxy.sh ev_$1/prof_proxy8 --exchange peer | tail -16 || exit 1
bash tools/kernel_profile.sh $T/c5_shard k_lloyd1 --n 62500000 --k 4096 --d 4 --dtype f16 --steps 10 --warmup 3 | tail -12 || exit 1
for N in 12500000 100000000; do
  timeout -k 10 200 python bench.py --split --no-cpu --fit-iters 0 --n $N > $T/split_graph_$N.json 2>&1 || { tail -20 $T/split_graph_$N.json; exit 1; }
  timeout -k 10 200 python bench.py --split --no-graph --no-cpu --fit-iters 0 --n $N > $T/split_eager_$N.json 2>&1 || { tail -20 $T/split_eager_$N.json; exit 1; }
  python3 -c "import json;g=json.loads(open('$T/split_graph_$N.json').read().strip().splitlines()[-1]);e=json.loads(open('$T/split_eager_$N.json').read().strip().splitlines()[-1]);print('split $N graph', round(g['ms_per_step'],5), 'eager', round(e['ms_per_step'],5), g['breakdown_ms_per_iter'], e['breakdown_ms_per_iter'])"
done
timeout -k 10 200 python bench.py --gpus 2 --backend gloo --n 20000000 --no-cpu --fit-iters 0 --steps 5 --warmup 2 > $T/gloo2.txt 2>&1 || { tail -20 $T/gloo2.txt; exit 1; }
timeout -k 10 200 python bench.py --gpus 3 --backend gloo --n 30000000 --no-cpu --fit-iters 0 --steps 5 --warmup 2 > $T/gloo3.txt 2>&1 || { tail -20 $T/gloo3.txt; exit 1; }
tail -1 $T/gloo3.txt | cut -c1-400
tail -1 $T/gloo2.txt | cut -c1-400
