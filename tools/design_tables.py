"""Print the measurement tables of DESIGN.md §6 and README.md from a final sweep's records (profiles/<prefix>_*):
the search kernels (rocprof average, HIP events, fp32-MFMA fraction recomputed from rocprof, PMC), the latency path
and the secondary rows.  Used to write those tables, so the documents quote the records verbatim.

    python tools/design_tables.py [--prefix r06z]
"""
import argparse
import csv
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "profiles")
MFMA_PEAK = 157.3e12
ROWS = [("c2", "configs[2] on 1 GPU, 65,536 roots"), ("s32k", "configs[2] shard N=2, 32,768 roots"),
        ("s16k", "configs[2] shard N=4, 16,384 roots"), ("b8192", "configs[2] shard N=8, 8,192 roots"),
        ("c1", "configs[1], 4,096 roots"), ("c3", "configs[3], 16,384 roots, S=200"),
        ("c4", "configs[4] on 1 GPU, 262,144 roots"), ("c4s8", "configs[4] shard N=8, 32,768 roots (7 disks, S=100)")]


def load(name):
    return json.load(open(os.path.join(P, name)))


def search_rows(px):
    out = []
    for t, name in ROWS:
        s, b = load(f"{px}_{t}_prof_summary.json"), load(f"{px}_bench_{t}.json")
        f, r = s["fused"], b["roofline"]
        tr = r["tree"]
        avg = f["avg_ns"] * 1e-6
        frac = r["flop_per_launch"] / (avg * 1e-3) / MFMA_PEAK
        fr = tr["binding"]["fracs"]
        out.append(f"| {name} | {r['kernel'].replace('mzh_', '').replace('_kernel', '')} | {avg:.3f} / "
                   f"{s['unprofiled']['kernel_ms_hip_events']:.3f} ms | {frac:.3f} | {f['mfma_busy_frac']:.3f} | "
                   f"{f['clock_ghz']:.2f} GHz | {f['hbm_bytes_per_launch'] / 1e9:.3g} GB | {f['l2_hit_rate']:.3f} | "
                   f"{fr['hbm']:.3f} / {fr['latency']:.3f} / {fr['issue']:.3f} ({tr['binding']['ceiling']}) | "
                   f"{tr['latency']['levels_per_sim']['max_group']:.2f} | {b['value']:.3g} |")
    return out


def one_kernel_avg_us(px, name="mzh_search_one_kernel<true, true, true>"):
    for row in csv.DictReader(open(os.path.join(P, f"{px}_one_kernel_stats.csv"))):
        if name in row["Name"]:
            return float(row["AverageNs"]) / 1e3, int(row["Calls"])
    return None, 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prefix", default="r06z")
    px = ap.parse_args().prefix
    print("\n".join(search_rows(px)))
    d = load(f"{px}_bench_default.json")
    print(json.dumps({"default_line": {"value": d["value"], "frac": d["roofline"]["frac"],
                                       "cpu": d["cpu_baseline"]["value"], "predraw_ms": d["predraw"]["ms"],
                                       "build_id": d.get("build_id")}}))
    print(json.dumps({"one_kernel_run_mcts_us": one_kernel_avg_us(px)}))
    pr = load(f"{px}_one_probe.json")
    print(json.dumps({"one_probe": [(r["disks"], r["sims"], r["roots"], round(r["one_ms"], 3), round(r["coop_ms"], 3),
                                     r["identical"]) for r in pr["rows"]], "run_mcts": pr["run_mcts"]}))
    for f in ("selfplay_bench", "env_bench", "eval_bench", "train_bench"):
        rows = load(f"{px}_{f}.json")
        rows = rows if isinstance(rows, list) else rows.get("rows", [rows])
        print(f, json.dumps({r.get("leg"): r.get("value") for r in rows}))


if __name__ == "__main__":
    main()
