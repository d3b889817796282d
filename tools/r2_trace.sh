#!/bin/bash
# kernel timeline (durations + gaps) of the multi-GPU call sequence at a 12.5M shard and of config 3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tr
for cfg in "s12:--split --n 12500000" "c3:" "c3e:--no-graph"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr/$tag -o run -- python3 bench.py --no-cpu --fit-iters 0 --no-events $args > gpurun_out/tr/$tag.log 2>&1 || { tail -5 gpurun_out/tr/$tag.log; exit 1; }
  echo "== $tag"; python3 tools/trace_gaps.py gpurun_out/tr/$tag 40
done
