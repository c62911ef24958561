"""Copy one tools/gpu/sweep.sh run from gpurun_out/ into profiles/ under a round prefix, and merge its
PMC traffic entries into profiles/traffic_latest.json (entries of other workloads are kept; bench.py
reports an entry only for the build it was profiled on).

  python tools/collect_sweep.py r05f c2 b8192 ...
"""
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def main():
    prefix, tags = sys.argv[1], sys.argv[2:]
    for t in tags:
        ks = sorted(glob.glob(os.path.join(OUT, f"prof_{t}_trace", "*", "*_kernel_stats.csv")))
        if ks:
            shutil.copy(ks[-1], os.path.join(PROF, f"{prefix}_{t}_kernel_stats.csv"))
        for src, dst in ((f"traffic_{t}.json", f"{prefix}_{t}_prof_summary.json"),
                         (f"bench_{t}.json", f"{prefix}_bench_{t}.json")):
            if os.path.exists(os.path.join(OUT, src)):
                shutil.copy(os.path.join(OUT, src), os.path.join(PROF, dst))
        print(t, "kernel_stats" if ks else "-", os.path.exists(os.path.join(OUT, f"traffic_{t}.json")))
    new = os.path.join(OUT, "traffic_latest.json")
    if os.path.exists(new):
        cur_p = os.path.join(PROF, "traffic_latest.json")
        cur = json.load(open(cur_p)) if os.path.exists(cur_p) else {"entries": {}}
        add = json.load(open(new))
        cur["entries"].update(add.get("entries", {}))
        cur["what"] = add.get("what", cur.get("what"))
        json.dump(cur, open(cur_p, "w"), indent=1)
        print("merged", sorted(add.get("entries", {})))


if __name__ == "__main__":
    main()
