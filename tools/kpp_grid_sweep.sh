#!/bin/bash
# k-means++ eval/apply grid for the later centres (PCM_KPP_LATE_DIV: grid / div from centre PCM_KPP_LATE_C on)
for dv in 1 2 4 8; do
  PCM_KPP_LATE_DIV=$dv bash tools/kpp_prof.sh kg_$dv | sed "s/^/div=$dv /" | grep -v "call 0"
done
