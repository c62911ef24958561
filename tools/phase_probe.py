"""Phase probe: split the fused search time into tree work and MLP work (diagnostic only).

  full      mzh_search (MLP mode)                    B roots x S sims
  tree      mzh_search_replay (same tree, no MLP)    B roots x S sims, recorded-style outputs
  mlp_rec   mzh_recurrent_inference over B rows      x S  (one launch per simulation step)
  mlp_ini   mzh_initial_inference over B rows
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return float(np.median(ts))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--roots", type=int, default=8192)
    p.add_argument("--sims", type=int, default=50)
    p.add_argument("--disks", type=int, default=4)
    p.add_argument("--kernel", default=None)
    a = p.parse_args()
    from bench import random_roots
    from muzero_hanoi_amd import engine, rng
    from muzero_hanoi_amd.networks import MuZeroNet

    N, S, B = a.disks, a.sims, a.roots
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = MuZeroNet(3 * N, 6, 0.002, "cpu", TD_return=True)
    eng = engine.Engine(N, S, B, 33)
    eng.load_weights(engine.flat_weights(net.state_dict()))
    obs = torch.from_numpy(random_roots(N, B, 1)).to(dev)
    noise, tie, u = (torch.from_numpy(x).to(dev) for x in rng.synthetic_draws(B, deterministic=False, alpha=0.25, seed=1))
    out = eng.alloc_search_outputs(B, S)
    res = {}
    res["full_ms"] = timeit(lambda: eng.search(S, obs=obs, tie_idx=tie, noise=noise, action_u=u, out=out, kernel=a.kernel))
    # replay inputs shaped like real network outputs
    g = np.random.default_rng(0)
    pi = g.dirichlet(np.ones(6), size=(B, S)).astype(np.float32)
    rp = dict(root_pi=torch.from_numpy(g.dirichlet(np.ones(6), size=B).astype(np.float32)).to(dev),
              pi=torch.from_numpy(pi).to(dev),
              reward=torch.from_numpy(g.normal(0, 0.05, (B, S)).astype(np.float32)).to(dev),
              value=torch.from_numpy(g.normal(0, 1, (B, S)).astype(np.float32)).to(dev))
    res["tree_ms"] = timeit(lambda: eng.search(S, replay=rp, tie_idx=tie, noise=noise, action_u=u, out=out, kernel=a.kernel))
    h = torch.rand((B, 64), device=dev)
    act = torch.randint(0, 6, (B,), dtype=torch.int32, device=dev)
    res["mlp_rec_one_ms"] = timeit(lambda: eng.recurrent_inference(h, act))
    res["mlp_ini_one_ms"] = timeit(lambda: eng.initial_inference(obs))
    res["mlp_rec_x_sims_ms"] = res["mlp_rec_one_ms"] * S
    flop = B * 203776
    res["mlp_rec_tflops"] = flop / (res["mlp_rec_one_ms"] * 1e-3) / 1e12
    res["full_tflops"] = B * (S * 203776 + 2 * (768 * N + 59136)) / (res["full_ms"] * 1e-3) / 1e12
    res["config"] = dict(B=B, S=S, N=N)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
