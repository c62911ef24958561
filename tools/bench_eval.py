"""Batched evaluation metrics: acting_ablations.get_results
(acting_experiments/acting_ablations.py:72-128) over a batch of start states and several search
budgets -- episodes played to the goal or max_steps, (steps - optimal) per start with the optimal
count from hanoi_solver (env/hanoi_utils.py:4-26), and the illegal-move rate
(illegal_move_rate_comparison.py:27-50) -- plus the hanoi_solver kernel alone.

Legs:
  evaluate     selfplay.evaluate on the GPU: every start of a budget in one lockstep batch, each
               episode its own agent (MinMaxStats carried over its decisions)
  solver       device hanoi_solver over 2^20 random states (N=7) vs the C restatement on one host
               core (bench.cpu_baseline_solver, bounded sample)

  python tools/bench_eval.py [--starts 4096] [--budgets 1,5,10,25,50]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--starts", type=int, default=4096)
    ap.add_argument("--budgets", default="1,5,10,25,50")
    ap.add_argument("--disks", type=int, default=3)
    ap.add_argument("--max-steps", type=int, default=200)
    ap.add_argument("--solver-states", type=int, default=1 << 20)
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from muzero_hanoi_amd.engine import hanoi_solver_batch
    from muzero_hanoi_amd.networks import MuZeroNet
    from muzero_hanoi_amd.selfplay import evaluate

    from bench import cpu_baseline_solver

    recs = []
    torch.manual_seed(1)
    net = MuZeroNet(3 * a.disks, 6, 0.002, "cuda", TD_return=True).to("cuda")
    budgets = [int(x) for x in a.budgets.split(",")]
    starts = np.random.default_rng(0).integers(0, 3 ** a.disks - 1, size=a.starts)
    evaluate(net, a.disks, budgets[:1], start_idx=starts[:64], max_steps=a.max_steps)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = evaluate(net, a.disks, budgets, start_idx=starts, max_steps=a.max_steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    recs.append({"leg": "evaluate", "metric": "evaluate_seconds", "value": dt, "unit": "s",
                 "episodes": a.starts * len(budgets), "episodes_per_sec": a.starts * len(budgets) / dt,
                 "results": [{"n_sims": n, "mean_steps_over_optimal": e, "illegal_rate_mean": il, "illegal_rate_sem": se}
                             for (n, e), (_, il, se) in zip(out["data"], out["illegal"])],
                 "config": {"workload": f"hanoi{a.disks}_maxsteps{a.max_steps}", "starts": a.starts,
                            "budgets": budgets, "network": "random-init MuZeroNet(TD_return=True)"}})
    print(json.dumps(recs[-1]), flush=True)

    n = 7
    g = np.random.default_rng(1)
    st = g.integers(0, 3, size=(a.solver_states, n)).astype(np.uint8)
    dst = torch.from_numpy(st).cuda()
    hanoi_solver_batch(n, dst)
    torch.cuda.synchronize()
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        out = hanoi_solver_batch(n, dst)
    torch.cuda.synchronize()
    gpu = reps * a.solver_states / (time.perf_counter() - t0)
    ref, cpu = cpu_baseline_solver(st, a.cpu_seconds)
    k = len(ref)
    same = bool(np.array_equal(out[:k].cpu().numpy(), ref))
    recs.append({"leg": "solver", "metric": "hanoi_solver_states_per_sec", "value": gpu, "unit": "states/s",
                 "cpu_baseline": {"value": cpu, "unit": "states/s", "cores": 1, "kind": "port",
                                  "sample": f"{k} states through oracle/mzh_oracle.c via ctypes"},
                 "matches_oracle_on_sample": same,
                 "config": {"workload": f"hanoi{n}_random_states", "states": a.solver_states}})
    print(json.dumps(recs[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(recs, f, indent=1)


if __name__ == "__main__":
    main()
