"""Latency kernel vs cooperative kernel by batch size (the crossover behind mzh_api.hip kOneMaxRoots), and the
drop-in run_mcts call broken into kernel and host time.

    python tools/one_probe.py [--out profiles/r06_one_probe.json]

Per (disks, sims, roots): HIP-event time of one mzh_search launch (median of 7 after 2 warm-ups) for the
latency kernel ("one") and the cooperative kernel ("coop"), random non-goal roots, T=1 stochastic draws,
random-init MuZeroNet(TD_return=True) weights; then MCTS.run_mcts (N=3, S=25, the training config) timed
end to end on the host and its kernel alone.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, reps=7, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    return float(np.median([s.elapsed_time(e) for s, e in ev]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import bench
    from muzero_hanoi_amd import engine, rng
    from muzero_hanoi_amd.networks import MuZeroNet

    rows = []
    for n, S in ((3, 25), (4, 50)):
        torch.manual_seed(0)
        net = MuZeroNet(3 * n, 6, 0.002, "cpu", TD_return=True)
        flat = engine.flat_weights(net.state_dict())
        Bmax = 4096
        eng = engine.Engine(n, S, Bmax, 33)
        eng.load_weights(flat)
        obs_all = torch.from_numpy(bench.random_roots(n, Bmax, 0)).cuda()
        noise, tie, u = rng.synthetic_draws(Bmax, deterministic=False, alpha=0.25, seed=0)
        noise, tie, u = (torch.from_numpy(x).cuda() for x in (noise, tie, u))
        for B in (1, 4, 16, 64, 256, 512, 1024, 2048, 4096):
            row = {"disks": n, "sims": S, "roots": B}
            outs = {}
            for k in ("one", "coop"):
                out = eng.alloc_search_outputs(B, S)
                fn = lambda: eng.search(S, obs=obs_all[:B], tie_idx=tie[:B], noise=noise[:B], action_u=u[:B],
                                        temperature=1.0, out=out, kernel=k)
                row[f"{k}_ms"] = timed(fn)
                row[f"{k}_kernel"] = out["_plan"]["kernel"]
                outs[k] = {kk: v.cpu() for kk, v in out.items() if not kk.startswith("_")}
            row["identical"] = all(torch.equal(outs["one"][kk], outs["coop"][kk]) for kk in ("visits", "root_q",
                                                                                         "action", "sel_steps"))
            row["one_sims_per_s"] = B * S / (row["one_ms"] * 1e-3)
            rows.append(row)
            print(json.dumps(row), flush=True)
        eng.close()

    # the drop-in: MCTS.run_mcts, N = 3, S = 25, as Muzero._play_game calls it
    from muzero_hanoi_amd.mcts import MCTS

    torch.manual_seed(0)
    net = MuZeroNet(9, 6, 0.002, "cuda", TD_return=True)
    m = MCTS(0.8, 0.25, 25, 256, "cuda")
    obs = bench.random_roots(3, 64, 5).astype(np.float64)
    np.random.seed(0)
    for i in range(20):
        m.run_mcts(obs[i % 64], net, 1.0, False)
    torch.cuda.synchronize()
    calls = 400
    t0 = time.perf_counter()
    for i in range(calls):
        m.run_mcts(obs[i % 64], net, 1.0, False)
    dt = (time.perf_counter() - t0) / calls
    dropin = {"what": "MCTS.run_mcts wall time per call (N=3, S=25, T=1 stochastic; the reference-order pre-draw, the "
                      "zero-copy staging record (mapped page-locked memory), the search launch, one stream sync)",
              "ms_per_call": dt * 1e3, "calls_per_s": 1.0 / dt}
    print(json.dumps(dropin), flush=True)
    if a.out:
        json.dump({"rows": rows, "run_mcts": dropin}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
