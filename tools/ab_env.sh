#!/bin/bash
# A/B of an environment switch on the config-3 bench line (whole fit included), alternating:
#   tools/ab_env.sh OUT VAR "v1 v2" REPS [pytest files...]
set -o pipefail
T=gpurun_out/$1; VAR=$2; VALS=$3; REPS=$4; shift 4; mkdir -p $T
export PYTHONUNBUFFERED=1
if [ $# -gt 0 ]; then
  timeout -k 10 500 python -u -m pytest "$@" -m gpu -x -q --timeout 200 --timeout-method thread > $T/pytest.txt 2>&1 || { tail -30 $T/pytest.txt; exit 1; }
  tail -1 $T/pytest.txt
fi
for r in $(seq $REPS); do for v in $VALS; do
  env $VAR=$v timeout -k 10 200 python bench.py --no-cpu --no-kpp --steps 20 > $T/b_${v}_$r.json 2> $T/b.err || { tail -20 $T/b.err; exit 1; }
  tail -1 $T/b_${v}_$r.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); f=d['fit']; print('$VAR=$v', 'step', round(d['ms_per_step'],4), 'layout', round(d['layout_ms'],3), 'fit warm', round(f['warm_ms'],3), 'cold', round(f['cold_ms'],3))"
done; done
