"""Summarise rocprofv3 outputs under gpurun_out/prof_* for the search kernel (newest run of each pass)."""
import collections
import csv
import glob
import json
import os
import sys

ROOT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
KERNEL = sys.argv[2] if len(sys.argv) > 2 else "mzh_wave_kernel<2"  # substring of the dominant kernel


def newest(pattern):
    f = sorted(glob.glob(os.path.join(ROOT, pattern)), key=os.path.getmtime)
    return f[-1] if f else None


out = {}
ks = newest("prof_trace/*/*_kernel_stats.csv")
if ks:
    for r in csv.DictReader(open(ks)):
        if KERNEL in r["Name"]:
            out["kernel"] = r["Name"]
            out["calls"] = int(r["Calls"])
            out["avg_ns"] = float(r["AverageNs"])
for p in ("hit", "fetch", "write", "sq"):
    f = newest(f"prof_{p}/*/*_counter_collection.csv")
    if not f:
        continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if KERNEL in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append((r["Dispatch_Id"], float(r["Counter_Value"])))
    for k, v in agg.items():  # sum over the per-XCD / per-SE rows of one dispatch, mean over dispatches
        per = collections.defaultdict(float)
        for d, x in v:
            per[d] += x
        out[k] = sum(per.values()) / len(per)
if "TCC_HIT_sum" in out:
    out["l2_hit_rate"] = out["TCC_HIT_sum"] / (out["TCC_HIT_sum"] + out["TCC_MISS_sum"])
if "FETCH_SIZE" in out:
    out["hbm_read_bytes_corrected"] = out["FETCH_SIZE"] * 1024 * 2  # KB; x2 gfx950 correction
if "WRITE_SIZE" in out:
    out["hbm_write_bytes"] = out["WRITE_SIZE"] * 1024
print(json.dumps(out, indent=1))
