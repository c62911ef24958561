"""Read the in-kernel phase stamps of the diagnostic build (libmzh_diag.so, -DMZH_STAMPS).
Phase ids: see MZH_STAMP(...) in csrc/mzh_device.h / mzh_search.hip.  s_memtime ticks of workgroup 0,
averaged per MLP step (recurrent kernel) and per simulation (search kernel)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MZH_LIB"] = os.environ.get("MZH_DIAG_LIB", os.path.join(ROOT, "muzero-hanoi_amd", "libmzh_diag.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from muzero_hanoi_amd import _lib, engine, rng  # noqa: E402
from muzero_hanoi_amd.networks import MuZeroNet  # noqa: E402

MLP = {0: "prologue", 1: "dyn0", 2: "bar+fetch", 3: "dyn2", 4: "bar+fetch", 5: "norm", 6: "rwd0", 7: "bar+fetch",
       8: "rwd2|pred4", 9: "pred4+pred3", 10: "bar+pol2/val2", 11: "bar+heads", 12: "bar"}
SEARCH = {16: "backup:latent+new-block stores", 17: "backup:value chain (lane 0)", 18: "backup:path updates",
          29: "backup:min-max reduce+set", 13: "select:setup (mm, tie load)", 14: "select:root level+prefetch",
          15: "select:level loop", 31: "select:bookkeeping+latent gather", 30: "select (own group)", 19: "bar->mlp", 20: "mlp", 21: "heads",
          22: "expand+backup", 23: "bar (select of the slowest group)"}


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    replay = "--replay" in sys.argv
    S = 50
    torch.manual_seed(0)
    net = MuZeroNet(12, 6, 0.002, "cpu", TD_return=True)
    eng = engine.Engine(4, S, B, 33)
    eng.load_weights(engine.flat_weights(net.state_dict()))
    L = _lib.lib()
    L.mzh_diag_stamps.argtypes = [ctypes.c_void_p]
    buf = np.zeros((8, 32), np.uint64)
    h = torch.rand((B, 64), device="cuda")
    a = torch.randint(0, 6, (B,), dtype=torch.int32, device="cuda")
    eng.recurrent_inference(h, a)
    torch.cuda.synchronize()
    L.mzh_diag_stamps(buf.ctypes.data)
    reps = 10
    for _ in range(reps):
        eng.recurrent_inference(h, a)
    torch.cuda.synchronize()
    L.mzh_diag_stamps(buf.ctypes.data)
    per = (buf / reps).astype(np.int64)
    out = {"mlp_step": {f"{k}:{v}": per[:4, k].tolist() for k, v in MLP.items()},
           "mlp_total": per[:4, 0:13].sum(1).tolist()}
    from bench import random_roots
    obs = torch.from_numpy(random_roots(4, B, 1)).cuda()
    noise, tie, u = (torch.from_numpy(x).cuda() for x in rng.synthetic_draws(B, deterministic=False, alpha=0.25, seed=1))
    rp = None
    if replay:  # network outputs drawn like bench.py's tree measurement
        g = np.random.default_rng(7)
        rp = dict(root_pi=torch.from_numpy(g.dirichlet(np.full(6, 20.0), size=B).astype(np.float32)).cuda(),
                  pi=torch.from_numpy(g.dirichlet(np.full(6, 20.0), size=(B, S)).astype(np.float32)).cuda(),
                  reward=torch.from_numpy(g.normal(0, 0.05, (B, S)).astype(np.float32)).cuda(),
                  value=torch.from_numpy(g.normal(0, 0.5, (B, S)).astype(np.float32)).cuda())
    run = lambda: eng.search(S, obs=None if replay else obs, replay=rp, tie_idx=tie, noise=noise, action_u=u)
    run()
    torch.cuda.synchronize()
    L.mzh_diag_stamps(buf.ctypes.data)
    run()
    torch.cuda.synchronize()
    L.mzh_diag_stamps(buf.ctypes.data)
    per = buf / S
    out["search_per_sim"] = {f"{k}:{v}": per[:4, k].tolist() for k, v in SEARCH.items()}
    out["search_per_sim_total"] = (per[:4, 19:24].sum(1) + per[:4, 30]).tolist()  # 16-18, 29 split 22
    lv = {24: "mem(block)", 25: "ucb", 26: "pick", 27: "path+shfl"}
    its = per[:4, 28] * S
    out["select_level_ticks"] = {f"{k}:{v}": (per[:4, k] * S / np.maximum(its, 1)).round().tolist() for k, v in lv.items()}
    out["select_levels_per_sim"] = (its / S).tolist()
    out["mlp_in_search_per_sim"] = {f"{k}:{v}": per[:4, k].tolist() for k, v in MLP.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
