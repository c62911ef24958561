"""Summarise one tools/prof.sh run (gpurun_out/prof_<tag>_*): per search kernel instantiation -- the
fused search (REPLAY = false) and its replay / tree-only instantiation (REPLAY = true) -- the
rocprofv3 average duration and the per-launch PMC values, HBM bytes corrected as
MI355X_MICROARCH.md prescribes (FETCH_SIZE x 2 on gfx950, WRITE_SIZE as is; both in KB).

  python tools/traffic.py gpurun_out TAG [--traffic-json profiles/traffic_latest.json]
"""
import collections
import csv
import glob
import json
import os
import sys


def newest(root, pattern):
    f = sorted(glob.glob(os.path.join(root, pattern)), key=os.path.getmtime)
    return f[-1] if f else None


def kind(name):
    """search kernels only: 'fused' or 'tree' by the REPLAY template argument"""
    if "mzh_wave_kernel<" not in name and "mzh_search_kernel<" not in name:
        return None
    args = name.split("<", 1)[1].split(">", 1)[0].split(",")
    return "tree" if args[1].strip() == "true" else "fused"


def summarise(root, tag, want=None):
    """want: {"fused": name, "tree": name} -- the instantiations the bench line reports; any other
    search-kernel instantiation the command launched (e.g. the minmax_in leg's MMIN = true) is listed
    under "other" with its stats and kept out of the fused / tree figures"""
    out = {"fused": {}, "tree": {}, "other": {}}
    want = want or {}

    def slot(name):
        k = kind(name)
        if k and want.get(k) and want[k] not in name:
            return "other"
        return k

    ks = newest(root, f"prof_{tag}_trace/*/*_kernel_stats.csv") or newest(root, f"prof_{tag}_trace/*_kernel_stats.csv")
    if ks:
        for r in csv.DictReader(open(ks)):
            k = slot(r["Name"])
            if k == "other":
                out["other"][r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
            elif k:
                out[k].update(kernel=r["Name"], calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]))
    for p in ("hit", "fetch", "write", "sq"):
        f = newest(root, f"prof_{tag}_{p}/*/*_counter_collection.csv") or newest(root, f"prof_{tag}_{p}/*_counter_collection.csv")
        if not f:
            continue
        agg = {"fused": collections.defaultdict(lambda: collections.defaultdict(float)),
               "tree": collections.defaultdict(lambda: collections.defaultdict(float))}
        for r in csv.DictReader(open(f)):
            k = slot(r["Kernel_Name"])
            if k in agg:  # sum the per-XCD / per-SE rows of one dispatch
                agg[k][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for k in agg:
            for c, per in agg[k].items():
                out[k][c] = sum(per.values()) / len(per)  # mean over dispatches
    for k, d in out.items():
        if k == "other":
            continue
        if "TCC_HIT_sum" in d:
            d["l2_hit_rate"] = d["TCC_HIT_sum"] / (d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
        if "FETCH_SIZE" in d:
            d["hbm_read_bytes_corrected"] = d["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in d:
            d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
        if "hbm_read_bytes_corrected" in d and "hbm_write_bytes" in d:
            d["hbm_bytes_per_launch"] = d["hbm_read_bytes_corrected"] + d["hbm_write_bytes"]
        if "SQ_INSTS_MFMA" in d and "GRBM_GUI_ACTIVE" in d and "avg_ns" in d:
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs; 1024 SIMDs, 32 cycles per 16x16x4 f32 MFMA
            cyc = d["GRBM_GUI_ACTIVE"] / 8
            d["clock_ghz"] = cyc / d["avg_ns"]
            d["mfma_busy_frac"] = d["SQ_INSTS_MFMA"] * 32 / (cyc * 1024)
            if "SQ_ACTIVE_INST_ANY" in d:
                # the issue ceiling: cycles some wave of a SIMD issued (SQ_ACTIVE_INST_ANY counts quad-cycles per
                # wave, summed over waves) over the SIMDs' cycles -- exact at one wave per SIMD, an upper bound
                # with two (overlapping issue of the pair is counted twice; bench.py labels it so)
                d["issue_frac"] = d["SQ_ACTIVE_INST_ANY"] * 4 / (cyc * 1024)
        if "SQ_WAIT_ANY" in d and "SQ_WAVE_CYCLES" in d:
            d["waitcnt_frac"] = d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"]  # wave cycles parked in s_waitcnt
    return out


def bench_line(path):
    """the last JSON line of a bench.py stdout capture (None if absent)"""
    if not os.path.exists(path):
        return None
    for line in reversed(open(path).read().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            try:
                return json.loads(line)
            except ValueError:
                continue
    return None


def main():
    """python tools/traffic.py gpurun_out TAG [--traffic-json PATH]: print the summary of the
    profiled bench command (tools/prof.sh TAG) beside the same command's un-profiled bench line on the
    same box; with --traffic-json, record the fused / tree kernels' PMC bytes under the workload key
    the PROFILED bench line itself looked up (roofline.traffic_source.key), stamped with the build id
    that run printed -- refused if the profiled and un-profiled runs, or this checkout, disagree on it"""
    import argparse

    sys.path.insert(0, ROOT)

    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("tag")
    ap.add_argument("--traffic-json", default=None)
    ap.add_argument("--expect-build", default=None,
                    help="build id the profiled run must report (default: the checked-out sources' hash)")
    a = ap.parse_args()
    prof = bench_line(os.path.join(a.root, f"prof_{a.tag}_trace.log"))
    plain = bench_line(os.path.join(a.root, f"prof_{a.tag}_plain.json"))
    ref = prof or plain
    want = None
    if ref is not None:
        want = {"fused": ref["roofline"]["kernel"], "tree": (ref["roofline"].get("tree") or {}).get("kernel")}
    out = summarise(a.root, a.tag, want)
    if plain is not None:
        r = plain["roofline"]
        out["unprofiled"] = {
            "build_id": plain.get("build_id"), "kernel": r["kernel"], "kernel_ms_hip_events": r["kernel_ms"],
            "ms_per_step": plain["ms_per_step"], "frac": r["frac"],
            "tree_kernel_ms_hip_events": (r.get("tree") or {}).get("kernel_ms"),
            "what": "the same bench command without rocprofv3, same box and build, run just before the profiled passes"}
        f = out["fused"]
        if f.get("avg_ns"):
            out["unprofiled"]["rocprof_over_hip_events"] = f["avg_ns"] * 1e-6 / r["kernel_ms"]
    if prof is not None:
        out["profiled_bench"] = {"build_id": prof.get("build_id"), "kernel": prof["roofline"]["kernel"],
                                 "key": prof["roofline"]["traffic_source"]["key"]}
    print(json.dumps(out, indent=1))
    if a.traffic_json:
        if prof is None:
            raise SystemExit("no bench line in the profiled run's log: nothing to key the entry on")
        if a.expect_build is None:
            from muzero_hanoi_amd import build as _build

            a.expect_build = _build.source_hash()
        bid = prof.get("build_id")
        if bid != a.expect_build or (plain is not None and plain.get("build_id") != bid):
            raise SystemExit(f"refusing to record: profiled build {bid}, un-profiled "
                             f"{plain.get('build_id') if plain else None}, expected {a.expect_build}")
        f, t = out["fused"], out["tree"]
        if f.get("kernel") and prof["roofline"]["kernel"] not in f["kernel"]:
            raise SystemExit(f"the profiled kernel {f['kernel']} is not the bench's {prof['roofline']['kernel']}")
        key = prof["roofline"]["traffic_source"]["key"]
        doc = json.load(open(a.traffic_json)) if os.path.exists(a.traffic_json) else {}
        entries = doc.get("entries", {})
        entries[key] = {
            "build_id": bid, "kernel": f.get("kernel"), "avg_ns": f.get("avg_ns"),
            "hbm_bytes_per_launch": f.get("hbm_bytes_per_launch"),
            "read_bytes_corrected": f.get("hbm_read_bytes_corrected"), "write_bytes": f.get("hbm_write_bytes"),
            "l2_hit_rate": f.get("l2_hit_rate"), "mfma_busy_frac": f.get("mfma_busy_frac"),
            "clock_ghz": f.get("clock_ghz"),
            "tree_kernel": t.get("kernel"), "tree_avg_ns": t.get("avg_ns"),
            "tree_hbm_bytes_per_launch": t.get("hbm_bytes_per_launch"),
            "tree_read_bytes_corrected": t.get("hbm_read_bytes_corrected"), "tree_write_bytes": t.get("hbm_write_bytes"),
            "tree_issue_frac": t.get("issue_frac"), "tree_waitcnt_frac": t.get("waitcnt_frac"),
            "issue_frac": f.get("issue_frac"),
            "unprofiled_kernel_ms": (out.get("unprofiled") or {}).get("kernel_ms_hip_events"),
            "source": f"tools/prof.sh TAG={a.tag} + tools/traffic.py: rocprofv3 --kernel-trace --stats and separate "
                      "--pmc passes of the bench command; FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, "
                      "per-dispatch sums, mean over dispatches; key and build id from the profiled bench line"}
        json.dump({"what": "per-launch HBM bytes (PMC) of the bench workloads, keyed by bench.traffic_key; "
                           "bench.py reports an entry only when its build_id is the running library's",
                   "entries": entries}, open(a.traffic_json, "w"), indent=1)
        print("recorded", key, file=sys.stderr)


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if __name__ == "__main__":
    main()
