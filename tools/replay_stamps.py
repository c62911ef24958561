"""Phase stamps of the device replay draw (diagnostic build, MZH_LIB=muzero-hanoi_amd/libmzh_diag.so):
s_memtime (shader-clock ticks) after the np.sum phase (full buffers, partial buffer), the validity / exactness pass +
scan, the cdf pass, the cdf sample, the search and the gather, for the reference's buffer (50,000) and
batch (256).  Median over 50 launches.

    MZH_LIB=muzero-hanoi_amd/libmzh_diag.so python tools/replay_stamps.py [--n 50000] [--m 256]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from muzero_hanoi_amd import _lib  # noqa: E402

PHASES = ["full_buffers", "partial_buffer", "pass1_scan", "cdf_pass", "cdf_sample", "search", "gather"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50000)
    ap.add_argument("--m", type=int, default=256)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    n, m, U, A, d = a.n, a.m, 5, 6, 9
    g = np.random.default_rng(0)
    dev = "cuda"
    prio = torch.from_numpy((g.random(n) + 0.05).astype(np.float32)).to(dev)
    cdf = torch.empty(n, dtype=torch.float64, device=dev)
    src = [torch.zeros((n, d), device=dev), torch.zeros((n, U), device=dev),
           torch.zeros((n, U), dtype=torch.int64, device=dev), torch.zeros((n, U, A), device=dev),
           torch.zeros((n, U), device=dev)]
    out = [torch.empty((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev) for t in src]
    u = torch.from_numpy(g.random(m)).to(dev)
    indx = torch.empty(m, dtype=torch.int64, device=dev)
    status = torch.zeros(16, dtype=torch.int32, device=dev)
    r = _lib.ReplayArgs(n=n, m=m, d_state=d, U=U, A=A)
    r.prio, r.u, r.cdf, r.indx, r.status = prio.data_ptr(), u.data_ptr(), cdf.data_ptr(), indx.data_ptr(), status.data_ptr()
    r.states, r.rwds, r.actions, r.pi, r.returns = (t.data_ptr() for t in src)
    r.out_states, r.out_rwds, r.out_actions, r.out_pi, r.out_returns = (t.data_ptr() for t in out)
    rows = []
    for _ in range(60):
        _lib.check(_lib.lib().mzh_replay_sample(ctypes.byref(r), _lib.stream_handle()), "mzh_replay_sample")
        torch.cuda.synchronize()
        rows.append(status.cpu().numpy()[2:10].astype(np.int64))
    t = np.median(np.array(rows[10:]), axis=0)  # cumulative ticks at the end of each phase
    res = {"n": n, "m": m, "clock": "s_memtime ticks (shader clock)",
           "phase_ticks": {ph: float(t[i + 1] - t[i]) for i, ph in enumerate(PHASES)},
           "total_ticks": float(t[7]), "build_id": _lib.build_id()}
    print(json.dumps(res))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
