"""Summarise rocprofv3 --pmc output (rocpd .db or *counter_collection.csv) for
one kernel: mean per dispatch over the dispatches after the first (warm-up).

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half
the bytes of a wide (16 B/lane) coalesced streaming read -> x2.
usage: python tools/pmc_summary.py KERNEL_SUBSTR DIR [DIR ...]
"""
import csv
import glob
import os
import json
import sqlite3
import sys
from collections import defaultdict


def load_db(path, kernel):
    per = defaultdict(lambda: defaultdict(float))
    c = sqlite3.connect(path)
    q = "select dispatch_id, counter_name, value, start, end from counters_collection where kernel_name like ?"
    for did, name, val, st, en in c.execute(q, (f"%{kernel}%",)):
        per[did][name] += float(val)
        per[did]["_ns"] = en - st
    return per


def load_csv(paths, kernel):
    per = defaultdict(lambda: defaultdict(float))
    for p in paths:
        for r in csv.DictReader(open(p)):
            if kernel in r["Kernel_Name"]:
                d = int(r["Dispatch_Id"])
                per[d][r["Counter_Name"]] += float(r["Counter_Value"])
                per[d]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return per


def main():
    kernel, dirs = sys.argv[1], sys.argv[2:]
    agg = defaultdict(list)
    for d in dirs:
        dbs = glob.glob(f"{d}/**/*.db", recursive=True)
        per = load_db(dbs[0], kernel) if dbs else load_csv(glob.glob(f"{d}/**/*counter_collection.csv",
                                                                      recursive=True), kernel)
        ids = sorted(per)[1:]
        last = int(os.environ.get("PMC_LAST", "0"))   # only the last N dispatches (e.g. late k-means++ steps)
        for i in (ids[-last:] if last > 0 else ids):
            for k, v in per[i].items():
                agg[k].append(v)
    out = {k: sum(v) / len(v) for k, v in agg.items()}
    if "FETCH_SIZE" in out:
        out["hbm_read_bytes_corrected"] = out["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in out:
        out["hbm_write_bytes"] = out["WRITE_SIZE"] * 1024
    if "GRBM_GUI_ACTIVE" in out and out.get("_ns"):
        out["clock_GHz"] = out["GRBM_GUI_ACTIVE"] / 8 / out["_ns"]   # summed over the 8 XCDs
    if "SQ_WAVE_CYCLES" in out:   # fractions of the waves' (quad-)cycles
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
            if k in out:
                out["frac_" + k] = out[k] / out["SQ_WAVE_CYCLES"]
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
