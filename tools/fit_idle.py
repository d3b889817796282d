"""GPU idle time inside the last whole fit of a bench kernel trace (from its
k_bbox_partial to the k_label after it + the label gathers), and the gaps
over 8 us.  usage: python tools/fit_idle.py TRACE_DIR"""
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
lab = [i for i, r in enumerate(rows) if "k_label" in r["Kernel_Name"]]
bb = [i for i, r in enumerate(rows) if "k_bbox_partial" in r["Kernel_Name"]]
end = min(lab[-1] + 3, len(rows) - 1)
start = max(i for i in bb if i < lab[-1])
seg = rows[start:end + 1]
t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1e3
print(f"fit span {(t1 - t0) / 1e3:.1f} us, busy {busy:.1f}, idle {(t1 - t0) / 1e3 - busy:.1f}, kernels {len(seg)}")
prev = None
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if prev is not None and s - prev > 8000:
        print(f"  gap {(s - prev) / 1e3:6.1f} us before {r['Kernel_Name'].split('(')[0][-45:]}")
    prev = e
