#!/bin/bash
# Calibration (GPU box): streaming probes + assign-kernel ablation builds.
mkdir -p gpurun_out/calib
[ -n "$PROBE" ] && { timeout -k 10 60 ./tools/stream_probe > gpurun_out/calib/stream.txt 2>&1 || exit 1; }


for v in "$@"; do
  PCM_SO=$PWD/tools/variants/lib_$v.so timeout -k 10 120 python bench.py --no-cpu --steps 20 --warmup 3 > gpurun_out/calib/$v.txt 2>&1 || { tail -5 gpurun_out/calib/$v.txt; exit 1; }
  echo "$v $(tail -1 gpurun_out/calib/$v.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(r["avg_launch_ms"]*1e3,1), "us", round(r["achieved"]), "GB/s step_ms", round(d["ms_per_step"],3), {k: round(v*1e3,1) for k, v in d["breakdown_ms_per_iter"].items()})')"
done
