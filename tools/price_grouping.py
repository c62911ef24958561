"""Price depth-aware lockstep grouping of roots on the CPU, no GPU time.

Every lockstep group of the search kernels -- a workgroup of the cooperative kernel (16 or 32 roots),
a wave of the wave kernels (16 or 32 roots) -- waits each simulation for its DEEPEST root's dependent
block loads (MCTS/node.py:72-88 per level, MCTS/mcts.py:80-86).  Roots are independent, so any
permutation of roots into groups gives the same outputs; this tool asks which permutation shortens
the chain, from the C oracle's per-simulation selection depths on bench.py's own inputs
(tests/golden/gen_fullbatch.py: the same roots and reference-order draws).

    python tools/price_grouping.py [--tags c1_4096 c2_shard7of8 c2_65536] [--max-roots 16384]

For each ordering it reports, per group of G consecutive roots, the lockstep levels
L_g = sum_s max_{r in g} (depth(r, s) - 1) (what the kernels count in mzh_search_args.lockstep_levels):
  - the mean over groups (total chain work) and
  - the max over groups (the launch's makespan when there is one group per CU or SIMD slot, which is
    the case for every BASELINE workload: 256 workgroups at 4,096 / 8,192 roots, 2 waves per SIMD at
    65,536),
next to the per-root mean and the single deepest root (a floor no grouping can beat).
Writes profiles/r06_grouping_price.json.
"""
import argparse
import json
import multiprocessing as mp
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

GROUP = {"c1_4096": [16], "c2_shard7of8": [32], "c2_65536": [32, 16], "c3_16384": [16]}


def _chunk(args):
    n, S, obs, noise, tie, u, det = args
    import gen_fullbatch as gf
    from oracle import oracle

    flat, sup = gf.weights(n)
    r = oracle.search(n, S, obs, flat=flat, support=sup, noise=noise, tie_idx=tie, action_u=u, temperature=1.0,
                      deterministic=det, discount=0.8, depths=True)
    return r["depths"], r["sel_steps"]


def depths_for(tag, max_roots, procs):
    import gen_fullbatch as gf

    n, GB, S, W, rk, seed, det = gf._spec(tag)
    obs, noise, tie, u = gf.inputs(tag)
    B = min(len(obs), max_roots)
    step = 256
    sl = lambda x, i: None if x is None else x[i:i + step]
    jobs = [(n, S, obs[i:min(B, i + step)], sl(noise, i), tie[i:min(B, i + step)], sl(u, i), det)
            for i in range(0, B, step)]
    with mp.get_context("spawn").Pool(procs) as pool:
        parts = pool.map(_chunk, jobs)
    dep = np.concatenate([p[0] for p in parts])
    steps = np.concatenate([p[1] for p in parts])
    # the fixture's selection-step counts pin the restated run to bench.py's (every root)
    fx = np.load(os.path.join(ROOT, "tests", "golden", f"full_{tag}.npz"))
    assert np.array_equal(steps, fx["sel_steps"][:B].astype(np.int64)), "depths run differs from the fixture"
    assert np.array_equal(dep.sum(1), steps)
    state = np.argmax(obs[:B].reshape(B, n, 3), axis=2)  # obs[3i + s_i] = 1 (utils.py:9-25)
    sidx = (state * (3 ** np.arange(n - 1, -1, -1))).sum(1)  # env/hanoi.py:23-25 index order
    return dep - 1, sidx  # levels below the root, as the kernels count them


def group_levels(lv, order, G):
    """per group of G consecutive roots in `order`: sum over simulations of the group's deepest level"""
    B, S = lv.shape
    x = lv[order]
    pad = (-B) % G
    if pad:
        x = np.concatenate([x, np.zeros((pad, S), x.dtype)])
    return x.reshape(-1, G, S).max(1).sum(1)


def price(tag, lv, sidx, G):
    B, S = lv.shape
    tot = lv.sum(1)
    orders = {
        "index (today)": np.arange(B),
        "by root state": np.argsort(sidx, kind="stable"),
        "by total depth (oracle: not computable before the search)": np.argsort(-tot, kind="stable"),
        "by root state, then total depth (oracle)": np.lexsort((-tot, sidx)),
    }
    # dealt orders: roots ranked by a depth proxy and dealt round-robin over the B / G groups, so every group
    # holds one root of each depth stratum (spreads the deep roots instead of gathering them)
    ngr = -(-B // G)

    def dealt(rank):
        o = np.full(ngr * G, -1, np.int64)
        o[:B] = rank
        o = o.reshape(G, ngr).T.ravel()
        return o[o >= 0] if B % G == 0 else o  # (B % G != 0: not a BASELINE shape)

    orders["dealt by total depth (oracle)"] = dealt(np.argsort(-tot, kind="stable"))
    # a proxy known before the search: the depth of the root's first k simulations (a short pre-search)
    for k in (5, 10):
        orders[f"dealt by the first {k} simulations' depth"] = dealt(np.argsort(-lv[:, :k].sum(1), kind="stable"))
    # a balanced order: states sorted by their mean depth, then dealt so that every group holds roots of
    # one state where possible (same as "by root state" up to the order of the states)
    st_mean = np.array([tot[sidx == k].mean() if (sidx == k).any() else 0 for k in range(sidx.max() + 1)])
    orders["by root state, states by mean depth"] = np.lexsort((np.arange(B), -st_mean[sidx]))
    res = {"roots": int(B), "sims": int(S), "group": G,
           "per_root_mean_levels_per_sim": float(lv.mean()),
           "deepest_root_levels_per_sim": float(tot.max() / S),
           "orders": {}}
    for name, o in orders.items():
        g = group_levels(lv, o, G)
        res["orders"][name] = {"mean_group_levels_per_sim": float(g.mean() / S),
                               "max_group_levels_per_sim": float(g.max() / S),
                               "p99_group_levels_per_sim": float(np.percentile(g, 99) / S)}
    # how much of the depth is fixed by the root state: per-state spread of the total depth
    within = np.array([tot[sidx == k].std() for k in np.unique(sidx)])
    res["total_depth_std_all"] = float(tot.std())
    res["total_depth_std_within_state_mean"] = float(within.mean())
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tags", nargs="*", default=["c1_4096", "c2_shard7of8", "c2_65536"])
    ap.add_argument("--max-roots", type=int, default=16384)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06_grouping_price.json"))
    a = ap.parse_args()
    procs = min(8, os.cpu_count() or 1)
    out = {}
    for tag in a.tags:
        lv, sidx = depths_for(tag, a.max_roots, procs)
        out[tag] = [price(tag, lv, sidx, G) for G in GROUP[tag]]
        for r in out[tag]:
            print(tag, "G", r["group"], "mean/root", round(r["per_root_mean_levels_per_sim"], 2), "deepest root",
                  round(r["deepest_root_levels_per_sim"], 2), flush=True)
            for k, v in r["orders"].items():
                print(f"   {k:60s} mean {v['mean_group_levels_per_sim']:.2f}  max {v['max_group_levels_per_sim']:.2f}")
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
