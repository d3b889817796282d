#!/bin/bash
mkdir -p gpurun_out/up
for cfg in "0 67108864" "1 200000000" "1 67108864" "1 33554432" "2 67108864" "2 33554432"; do
  set -- $cfg
  PCM_UNPERM=$1 PCM_UNPERM_WIN=$2 timeout -k 10 120 python tools/unperm_probe.py >> gpurun_out/up/log.txt 2>&1 || { tail -5 gpurun_out/up/log.txt; exit 1; }
  tail -1 gpurun_out/up/log.txt
done
