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
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
R = [(0, 10), (10, 50), (50, 200), (200, 600), (600, 1023)]
last = {}
for name in ["k_kpp_search", "k_kpp_eval", "k_kpp_apply"]:
    sel = [r for r in rows if name in r["Kernel_Name"]][-1023:]
    d = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in sel])
    last[name] = sel
    print(name, len(d), "mean", round(d.mean(), 1), " ".join(f"[{a}:{b}] {d[a:b].mean():.1f}" for a, b in R),
          "| total ms", " ".join(f"[{a}:{b}] {d[a:b].sum() / 1e3:.2f}" for a, b in R))
# wall per centre: start of search c -> start of search c+1 (kernels + gaps)
s = np.array([int(r["Start_Timestamp"]) for r in last["k_kpp_search"]]) / 1e3
w = np.diff(s)
print("wall per centre us", " ".join(f"[{a}:{b}] {w[a:min(b, len(w))].mean():.1f}" for a, b in R),
      "| total ms", " ".join(f"[{a}:{b}] {w[a:min(b, len(w))].sum() / 1e3:.2f}" for a, b in R))
PY
