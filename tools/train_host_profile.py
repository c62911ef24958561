"""Host-side split of one fused training update with the device replay draw (tools/bench_train.py's `fused`
leg): wall time of each host call of priority_sample / _update / update_priorities (the last one includes the
stream synchronisation, i.e. the GPU's remaining work), medians over the timed steps.

    python tools/train_host_profile.py [--steps 200] [--out F]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_train import synthetic_fill  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from muzero_hanoi_amd.muzero import Muzero

    torch.manual_seed(1)
    np.random.seed(1)
    mz = Muzero(env=None, s_space_size=9, n_action=6, discount=0.8, dirichlet_alpha=0.25, n_mcts_simulations=25,
                unroll_n_steps=5, batch_s=256, TD_return=True, n_TD_step=10, lr=0.002, buffer_size=50000,
                priority_replay=True, device="cuda", update_impl="fused")
    synthetic_fill(mz, 3, 50000)
    buf = mz.buffer
    rows = []
    for k in range(a.steps + 10):
        t0 = time.perf_counter()
        s, r, ac, p, ret, indx, w = buf.priority_sample(256)
        t1 = time.perf_counter()
        newp, vl, rl, pl = mz._update(s, r, ac, p, ret, w)
        t2 = time.perf_counter()
        buf.update_priorities(indx, newp)
        t3 = time.perf_counter()
        if k >= 10:
            rows.append((t1 - t0, t2 - t1, t3 - t2, t3 - t0))
    m = np.median(np.array(rows), axis=0) * 1e6
    res = {"us_priority_sample": m[0], "us_update_host": m[1], "us_update_priorities_incl_sync": m[2],
           "us_total": m[3], "steps": a.steps}
    print(json.dumps(res))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
