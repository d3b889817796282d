#!/bin/bash
# Tuning sweeps (GPU box), one preset per former one-off script:   tools/sweeps.sh PRESET [args]
#   tile       points per tile (PCM_TILE_CAP) at config 3 and on a 12.5M shard
#   cells      pruning-grid size (PCM_CELL_TARGET) on a 12.5M shard
#   drift      candidate-list reuse policy (PCM_DRIFT_KAPPA x PCM_DRIFT_ALPHA), 12.5M shard and config 3
#   slab       8-slab proxy vs grid density (PCM_CELL_TARGET) x candidate blocks per coarse cell (PCM_CAND_BPC_RT)
#   wpe LIB..  product build vs variant libraries tools/ab/lib_LIB.so (tools/build_variant.sh) at c3 / s12 / c5 shard
#   kppgrid    k-means++ late-step eval / apply grids (PCM_KPP_LATE_DIV, PCM_KPP_APPLY_DIV)
#   unperm     sorted-order labels -> row order variants (PCM_UNPERM x PCM_UNPERM_WIN, tools/unperm_probe.py)
#   split      multi-GPU call sequence on one GPU (an RCCL group of 1), eager and graph, at 12.5M and 100M
#   lpt        longest-list-first tile order (PCM_TILE_LPT): parity subset, config-5 shard + 8-slab, 12.5M split, config 3
#   pub        k_updlists' dedicated publisher block (PCM_UPD_PUB): parity subset, 8-slab A/B, a kernel trace
#   slabcap    8-slab proxy vs tile cap (PCM_TILE_CAP) and the tile order
# Output: gpurun_out/sw_PRESET/ and one summary line per run on stdout.
set -o pipefail
P=$1; shift
T=gpurun_out/sw_$P; mkdir -p $T
line() {  # name, json file, python expression over d
  tail -1 "$2" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', $3)"
}
run() {  # name, env assignments..., -- bench args...
  local name=$1; shift; local e=(); while [ "$1" != -- ]; do e+=("$1"); shift; done; shift
  env "${e[@]}" timeout -k 10 200 python bench.py --no-cpu --fit-iters 0 "$@" > $T/$name.txt 2>&1 || { tail -5 $T/$name.txt; exit 1; }
}
S12="--split --n 12500000"
B="round(d['ms_per_step']*1e3,1), 'us/iter assign', round(d['breakdown_ms_per_iter']['assign']*1e3,1)"
case $P in
  tile) for cap in 4096 2048 1536 1024; do
          run c3_$cap PCM_TILE_CAP=$cap --; line "c3 cap=$cap" $T/c3_$cap.txt "$B, 'tiles', d['config']['tiles']"
          run s12_$cap PCM_TILE_CAP=$cap -- $S12; line "s12 cap=$cap" $T/s12_$cap.txt "$B, 'tiles', d['config']['tiles']"
        done ;;
  cells) for t in 4096 8192 12288 16384; do
           run s12_$t PCM_CELL_TARGET=$t -- $S12
           line "target=$t" $T/s12_$t.txt "d['config']['cells'], d['config']['grid'], $B, 'cand', round(d['candidates']['mean'],2)"
         done ;;
  drift) for cfg in "0.05 2" "0.2 2" "0.5 2" "0.5 1.5" "1.0 2"; do set -- $cfg
           run s12_$1_$2 PCM_DRIFT_KAPPA=$1 PCM_DRIFT_ALPHA=$2 -- $S12
           run c3_$1_$2 PCM_DRIFT_KAPPA=$1 PCM_DRIFT_ALPHA=$2 --
           for w in s12 c3; do line "$w kappa=$1 alpha=$2" $T/${w}_$1_$2.txt "$B, 'cand', round(d['candidates']['mean'],2), 'rebuilds', d['candidates']['list_rebuilds'], '/', d['candidates']['iterations']"; done
         done ;;
  slab) for CT in 0 2048 8192 16384; do for BPC in 0 4 16; do
          E=(); [ $CT -gt 0 ] && E+=(PCM_CELL_TARGET=$CT); [ $BPC -gt 0 ] && E+=(PCM_CAND_BPC_RT=$BPC)
          env "${E[@]}" timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > $T/ct${CT}_b$BPC.json 2>&1 || { tail -5 $T/ct${CT}_b$BPC.json; exit 1; }
          line "cells=$CT bpc=$BPC" $T/ct${CT}_b$BPC.json "round(d['value'],1), 'us/rank', d['per_rank_us']['assign'], d['slabs'][1]['ncells']"
        done; done ;;
  wpe) for so in main "$@"; do
         E=(); [ $so != main ] && E+=(PCM_SO=tools/ab/lib_$so.so)
         run c3_$so "${E[@]}" --; line "$so c3" $T/c3_$so.txt "$B"
         run s12_$so "${E[@]}" -- $S12; line "$so s12" $T/s12_$so.txt "$B"
         run c5_$so "${E[@]}" -- --n 62500000 --k 4096 --d 4; line "$so c5" $T/c5_$so.txt "$B"
       done ;;
  kppgrid) for cfg in "1 4" "2 4" "4 4" "1 2" "1 8"; do set -- $cfg
             PCM_KPP_LATE_DIV=$1 PCM_KPP_APPLY_DIV=$2 bash tools/kpp_prof.sh sw_kppgrid/e$1_a$2 | sed "s/^/eval 1\/$1 apply 1\/$2 /" | grep -v "call 0"
           done ;;
  unperm) for cfg in "0 67108864" "1 200000000" "1 67108864" "1 33554432" "2 67108864" "2 33554432"; do set -- $cfg
            PCM_UNPERM=$1 PCM_UNPERM_WIN=$2 timeout -k 10 120 python tools/unperm_probe.py >> $T/log.txt 2>&1 || { tail -5 $T/log.txt; exit 1; }
            tail -1 $T/log.txt
          done ;;
  split) for n in 12500000 100000000; do for g in --no-graph ""; do
           run b_$n$g -- --split $g --n $n; line "n=$n $g" $T/b_$n$g.txt "round(d['ms_per_step']*1e3,1), 'us/iter', d['breakdown_ms_per_iter']"
         done; done ;;
  lpt) export PYTHONUNBUFFERED=1
       timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compressed.py tests/test_gpu_xchg.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -30 $T/pytest.txt; exit 1; }
       tail -1 $T/pytest.txt
       bash tools/ab_c5.sh sw_lpt/c5 PCM_TILE_LPT "0 -1" 2 || exit 1
       for v in 0 -1 0 -1; do
         PCM_TILE_LPT=$v timeout -k 10 200 python bench.py --split --no-cpu --fit-iters 0 --n 12500000 > $T/split_$v.json 2>&1 || { tail -5 $T/split_$v.json; exit 1; }
         line "split12.5M LPT=$v" $T/split_$v.json "round(d['ms_per_step']*1e3,1), d['breakdown_ms_per_iter']['assign']"
       done
       bash tools/ab_env.sh sw_lpt/c3 PCM_TILE_LPT "0 -1" 2 ;;
  pub) export PYTHONUNBUFFERED=1
       timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_xchg.py tests/test_gpu_multirank.py tests/test_gpu_crowded.py -m gpu -x -q --timeout 300 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -30 $T/pytest.txt; exit 1; }
       tail -1 $T/pytest.txt
       for r in 1 2; do for v in 0 1; do
         PCM_UPD_PUB=$v timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > $T/s8_${v}_$r.json 2>&1 || { tail -5 $T/s8_${v}_$r.json; exit 1; }
         line "slab8 PUB=$v" $T/s8_${v}_$r.json "'us/rank', round(d['value'],1), 'step', d['per_rank_us']['step'], 'bitwise', d['centres_bitwise_equal_single_engine']"
       done; done
       bash tools/prof_proxy.sh sw_pub/prof --exchange peer ;;
  slabcap) for r in 1 2; do for cfg in "4096 -1" "3072 1" "2048 1" "2048 0"; do set -- $cfg
             PCM_TILE_CAP=$1 PCM_TILE_LPT=$2 timeout -k 10 200 python bench.py --slab-of 8 --steps 20 --warmup 3 > $T/s8_$1_$2_$r.json 2>&1 || { tail -5 $T/s8_$1_$2_$r.json; exit 1; }
             line "cap $1 lpt $2" $T/s8_$1_$2_$r.json "'us/rank', round(d['value'],1), 'assign max', max(d['per_rank_us']['assign']), 'tiles', d['slabs'][0]['ntiles'], 'bitwise', d['centres_bitwise_equal_single_engine']"
           done; done ;;
  *) echo "unknown preset $P"; exit 2 ;;
esac
