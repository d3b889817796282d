#!/bin/bash
# which receive-buffer allocation / reader fence gives exact sums after buffer reuse
for alloc in 0 1 2; do for acq in 0 1; do
  echo "== alloc $alloc (0 uncached, 1 finegrained, 2 hipMalloc) acq $acq"
  PCM_XCHG_ALLOC=$alloc PCM_XCHG_ACQ=$acq timeout -k 10 100 python tools/xchg_diag.py 2>&1 | grep -v amdgpu.ids || exit 1
done; done
