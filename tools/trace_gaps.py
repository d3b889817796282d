"""Per-dispatch timeline from a rocprofv3 --kernel-trace CSV: mean duration of
each kernel over the last `n` dispatches of the hot loop and the idle gap
before it.  usage: python tools/trace_gaps.py TRACE_DIR [n]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
f = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tail = rows[-n:]
dur, gap = defaultdict(list), defaultdict(list)
prev_end = None
for r in tail:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    k = r["Kernel_Name"].split("(")[0][:60]
    dur[k].append((e - s) / 1e3)
    if prev_end is not None:
        gap[k].append((s - prev_end) / 1e3)
    prev_end = e
span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) / 1e3
print(f"last {n} dispatches span {span:.1f} us")
for k in dur:
    g = gap[k]
    print(f"{k:60s} n={len(dur[k]):3d} dur_us={sum(dur[k])/len(dur[k]):8.2f} gap_before_us={(sum(g)/len(g) if g else 0):7.2f}")
