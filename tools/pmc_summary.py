"""Summarise rocprofv3 outputs under gpurun_out/prof_* for the search kernel (newest run of each pass)."""
import collections
import csv
import glob
import json
import os
import sys

ROOT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"


def newest(pattern):
    f = sorted(glob.glob(os.path.join(ROOT, pattern)), key=os.path.getmtime)
    return f[-1] if f else None


out = {}
ks = newest("prof_trace/*/*_kernel_stats.csv")
if ks:
    for r in csv.DictReader(open(ks)):
        if "search_kernel" in r["Name"]:
            out["kernel"] = r["Name"]
            out["calls"] = int(r["Calls"])
            out["avg_ns"] = float(r["AverageNs"])
for p in ("hit", "fetch", "write", "sq"):
    f = newest(f"prof_{p}/*/*_counter_collection.csv")
    if not f:
        continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "search_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        out[k] = sum(v) / len(v)
if "TCC_HIT_sum" in out:
    out["l2_hit_rate"] = out["TCC_HIT_sum"] / (out["TCC_HIT_sum"] + out["TCC_MISS_sum"])
if "FETCH_SIZE" in out:
    out["hbm_read_bytes_corrected"] = out["FETCH_SIZE"] * 1024 * 2  # KB; x2 gfx950 correction
if "WRITE_SIZE" in out:
    out["hbm_write_bytes"] = out["WRITE_SIZE"] * 1024
print(json.dumps(out, indent=1))
