#!/bin/bash
# rocprofv3 kernel trace of one k-means++ seeding (config 3 shape) + per-step phase means
OUT=gpurun_out/${1:-kp}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/kpp_bench.py 100000000 1024 3 > $OUT/kpp.txt 2>&1 || { tail -20 $OUT/kpp.txt; exit 1; }
cat $OUT/kpp.txt | grep kmeans_plusplus
python3 - $OUT <<'PY'
import csv, glob, sys
import numpy as np
f = glob.glob(sys.argv[1] + "/trace/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for name in ["k_kpp_search", "k_kpp_eval", "k_kpp_apply"]:
    d = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if name in r["Kernel_Name"]])
    d = d[-1023:]
    print(name, len(d), "mean", round(d.mean(), 1), " ".join(f"[{a}:{b}] {d[a:b].mean():.1f}" for a, b in [(0, 10), (10, 50), (50, 200), (200, 600), (600, 1023)]))
PY
