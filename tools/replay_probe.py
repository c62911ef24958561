"""Replay (tree-only) search time by kernel at N=4, S=50: the plan the library picks against each forced kernel, the
visits compared with the default plan.  python tools/replay_probe.py"""
import sys, json, numpy as np, torch
sys.path.insert(0, '.')
import bench
from muzero_hanoi_amd import engine, rng
from muzero_hanoi_amd.networks import MuZeroNet
n, S = 4, 50
for B in (65536, 16384):
    torch.manual_seed(0)
    net = MuZeroNet(3 * n, 6, 0.002, "cpu", TD_return=True)
    eng = engine.Engine(n, S, B, 33); eng.load_weights(engine.flat_weights(net.state_dict()))
    noise, tie, u = (torch.from_numpy(x).cuda() for x in rng.synthetic_draws(B, deterministic=False, alpha=0.25, seed=0))
    g = np.random.default_rng(7)
    rp = dict(root_pi=torch.from_numpy(g.dirichlet(np.full(6, 20.0), size=B).astype(np.float32)).cuda(),
              pi=torch.from_numpy(g.dirichlet(np.full(6, 20.0), size=(B, S)).astype(np.float32)).cuda(),
              reward=torch.from_numpy(g.normal(0, 0.05, (B, S)).astype(np.float32)).cuda(),
              value=torch.from_numpy(g.normal(0, 0.5, (B, S)).astype(np.float32)).cuda())
    rp = dict(root_pi=rp["root_pi"], sim=engine.pack_replay(rp))
    res = {}
    for k in ("auto", "wave16", "wave", "coop"):
        out = eng.alloc_search_outputs(B, S)
        fn = lambda: eng.search(S, replay=rp, tie_idx=tie, noise=noise, action_u=u, temperature=1.0, out=out, kernel=k)
        fn(); torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(7)]
        for s_, e_ in ev:
            s_.record(); fn(); e_.record()
        torch.cuda.synchronize()
        res[k] = (float(np.median([s_.elapsed_time(e_) for s_, e_ in ev])), out["_plan"]["kernel"], out["visits"].cpu())
    base = res["auto"][2]
    print(json.dumps({"B": B, **{k: [round(v[0], 4), v[1], bool(torch.equal(v[2], base))] for k, v in res.items()}}))
    eng.close()
