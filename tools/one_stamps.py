"""In-kernel phase stamps of the latency kernel (mzh_search_one_kernel), diagnostic build only
(libmzh_diag.so: python -m muzero_hanoi_amd.build --diag).  s_memtime ticks per simulation of workgroup 0, per
wave, averaged over the launches: where one simulation of a one-root search goes.

    MZH_LIB=muzero-hanoi_amd/libmzh_diag.so python tools/one_stamps.py [--disks 3 --sims 25 --roots 1]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MZH_LIB"] = os.environ.get("MZH_DIAG_LIB", os.path.join(ROOT, "muzero-hanoi_amd", "libmzh_diag.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

PHASES = {1: "dyn0", 2: "bar1", 3: "dyn2+norm", 4: "bar2", 5: "rwd0|pol0+val0", 6: "bar3", 7: "rwd2/val2/pol2/bin32",
          8: "bar4", 9: "heads", 10: "backup", 11: "select", 12: "gather", 13: "bar5"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--disks", type=int, default=3)
    ap.add_argument("--sims", type=int, default=25)
    ap.add_argument("--roots", type=int, default=1)
    ap.add_argument("--launches", type=int, default=20)
    a = ap.parse_args()
    import bench
    from muzero_hanoi_amd import _lib, engine, rng
    from muzero_hanoi_amd.networks import MuZeroNet

    n, S, B = a.disks, a.sims, a.roots
    torch.manual_seed(0)
    net = MuZeroNet(3 * n, 6, 0.002, "cpu", TD_return=True)
    eng = engine.Engine(n, S, B, 33)
    eng.load_weights(engine.flat_weights(net.state_dict()))
    obs = torch.from_numpy(bench.random_roots(n, B, 0)).cuda()
    noise, tie, u = (torch.from_numpy(x).cuda() for x in rng.synthetic_draws(B, deterministic=False, alpha=0.25, seed=0))
    L = _lib.lib()
    L.mzh_diag_stamps_one.argtypes = [ctypes.c_void_p]
    buf = np.zeros((8, 32), np.uint64)
    run = lambda: eng.search(S, obs=obs, tie_idx=tie, noise=noise, action_u=u, temperature=1.0, kernel="one")
    run()
    torch.cuda.synchronize()
    L.mzh_diag_stamps_one(buf.ctypes.data_as(ctypes.c_void_p))
    sel = 0
    for _ in range(a.launches):
        o = run()
        sel += int(o["sel_steps"][0])
    torch.cuda.synchronize()
    L.mzh_diag_stamps_one(buf.ctypes.data_as(ctypes.c_void_p))
    per = buf.astype(np.float64) / (a.launches * S)
    sub = {}
    for name, base, parts in (("backup", 14, ("init+link", "value chain", "path updates", "root+minmax")),
                              ("select_level", 20, ("block load", "ucb", "pick", "take+path")),
                              ):
        cnt = float(buf[0, base + 4])
        if cnt:  # the groups the diagnostic build instruments (mzh_one.hip MZH_LSTAMP_FLUSH bases)
            sub[name] = {"count": cnt,
                         **{k: round(float(buf[0, base + i]) / cnt, 1) for i, k in enumerate(parts)}}
    out = {"disks": n, "sims": S, "roots": B, "sel_steps_per_sim": sel / (a.launches * S), "wave0_sub": sub,
           "ticks_per_sim": {f"wave{w}": {PHASES[k]: round(per[w, k], 1) for k in PHASES} for w in (0, 1, 2, 4)},
           "wave0_total": round(float(per[0, 1:14].sum()), 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
