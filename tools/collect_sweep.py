"""Copy one tools/gpu/sweep.sh run from gpurun_out/ into profiles/ under a round prefix, and merge its
PMC traffic entries into profiles/traffic_latest.json (re-derived from each tag's raw files; entries of other
workloads are kept; bench.py reports an entry only for the build it was profiled on).

  python tools/collect_sweep.py r05f c2 b8192 ...
"""
import glob
import json
import os
import shutil
import subprocess
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
    # the traffic entries are re-derived here from each tag's raw PMC files (tools/traffic.py records
    # the entry under its bench key with the build id of that run) rather than merged from
    # gpurun_out/traffic_latest.json: every gpurun call starts with an empty gpurun_out on the box, so
    # that file only ever holds the LAST call's tags (a sweep split over two calls lost its first half)
    cur_p = os.path.join(PROF, "traffic_latest.json")
    for t in tags:
        if glob.glob(os.path.join(OUT, f"prof_{t}_plain.json")):
            r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "traffic.py"), OUT, t,
                                "--traffic-json", cur_p], capture_output=True, text=True)
            print(t, r.stderr.strip().splitlines()[-1] if r.returncode == 0 and r.stderr.strip() else r.stderr.strip()[-200:])

if __name__ == "__main__":
    main()
