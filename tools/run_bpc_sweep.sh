#!/bin/bash
# k_step geometry sweep (candidate blocks per coarse cell x library variant), config 3
mkdir -p gpurun_out/f
for lib in t256 w4; do for b in 1 2 4; do
  PCM_CAND_BPC_RT=$b PCM_SO=3d-point-cloud-multiday-imagery_amd/libpcmkm_$lib.so timeout -k 10 120 python bench.py --no-cpu --fit-iters 0 > gpurun_out/f/b_${lib}_$b.txt 2>&1 || { tail -3 gpurun_out/f/b_${lib}_$b.txt; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/f/b_${lib}_$b.txt').read().strip().splitlines()[-1]); print('$lib bpc $b', round(d['ms_per_step'],4), d['breakdown_ms_per_iter'])"
done; done
for b in 1 2; do echo "== w4 bpc $b"; PCM_CAND_BPC_RT=$b timeout -k 10 60 python tools/step_timing2.py 3d-point-cloud-multiday-imagery_amd/libpcmkm_dbgw4.so 10 2>&1 | grep -v amdgpu.ids || exit 1; done
