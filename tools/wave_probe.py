"""Phase stamps of the wave kernel (diagnostic build libmzh_diag*.so, -DMZH_STAMPS): s_memtime
ticks per simulation for the 4 waves of workgroup 0, averaged over the S simulations."""
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

PH = {0: "select", 1: "mlp (value head)", 2: "head+backup", 3: "barrier", 4: "loop-top",
      10: "mlp: latent gather", 5: "mlp: dynamics chain", 6: "mlp: reward chain", 11: "mlp: reward head",
      7: "mlp: normalise + latent store", 8: "mlp: policy chain + softmax", 9: "mlp: value chain"}


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    S = 50
    torch.manual_seed(0)
    net = MuZeroNet(12, 6, 0.002, "cpu", TD_return=True)
    eng = engine.Engine(4, S, B, 33)
    eng.load_weights(engine.flat_weights(net.state_dict()))
    L = _lib.lib()
    L.mzh_diag_wave_stamps.argtypes = [ctypes.c_void_p]
    buf = np.zeros((8, 32), np.uint64)
    from bench import random_roots
    obs = torch.from_numpy(random_roots(4, B, 1)).cuda()
    noise, tie, u = (torch.from_numpy(x).cuda() for x in rng.synthetic_draws(B, deterministic=False, alpha=0.25, seed=1))
    eng.search(S, obs=obs, tie_idx=tie, noise=noise, action_u=u, kernel=os.environ.get("MZH_PROBE_KERNEL", "wave"))
    torch.cuda.synchronize()
    L.mzh_diag_wave_stamps(buf.ctypes.data)
    eng.search(S, obs=obs, tie_idx=tie, noise=noise, action_u=u, kernel=os.environ.get("MZH_PROBE_KERNEL", "wave"))
    torch.cuda.synchronize()
    L.mzh_diag_wave_stamps(buf.ctypes.data)
    per = buf[:8, :12] / S  # 8 waves (ping-pong workgroup); the 4-wave build leaves rows 4-7 zero
    out = {f"{k}:{v}": [round(x) for x in per[:, k]] for k, v in PH.items()}
    out["total"] = [round(x) for x in per.sum(1)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
