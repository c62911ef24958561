"""Training-update throughput: one `training_loop` update step =
`Buffer.priority_sample` + `Muzero._update` + `Buffer.update_priorities` (Muzero.py:123-140),
at the reference's TrainingConfig (training_main.py:15-34: Hanoi N=3, batch 256, 5 unroll steps,
TD returns, prioritised replay, buffer 50,000, lr 0.002), on synthetic transitions filling the
buffer.  Legs: the update on the host CPU (the reference's torch op sequence, parity-tested
against the reference's own fixtures), the eager update on the GPU, the HIP-graph update, and the
fused two-kernel HIP update (csrc/mzh_train.hip) with the prioritised draw and the priority write-back
on the device (Buffer(device_sampling=True), csrc/mzh_replay.hip; "fused-hostdraw": the same update with
the draw on the host in NumPy, as before round 6's device draw).

  python tools/bench_train.py [--legs cpu,gpu,graph,fused] [--steps K] [--warmup W] [--batch 256]

Prints one JSON line per leg: updates/s, samples/s (= transitions consumed per second) and
ms per update, plus the update-only time (sampling excluded).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def synthetic_fill(mz, n_disks, total, seed=0):
    g = np.random.default_rng(seed)
    U, A = mz.unroll_n_steps, mz.n_action
    chunk = 5000
    for a in range(0, total, chunk):
        T = min(chunk, total - a)
        st = g.integers(0, 3, (T, n_disks))
        states = np.zeros((T, 3 * n_disks), np.float32)
        states[np.arange(T)[:, None], np.arange(n_disks) * 3 + st] = 1
        rwds = np.where(g.random((T, U)) < 0.05, 100.0, np.where(g.random((T, U)) < 0.3, -0.1, 0.0))
        actions = g.integers(0, A, (T, U))
        pi = g.dirichlet(np.ones(A), size=(T, U))
        returns = g.normal(0.0, 20.0, (T, U))
        prios = g.random(T) + 0.05
        mz.buffer.add(states, rwds.astype(np.float32), actions, pi.astype(np.float32), returns.astype(np.float32),
                      prios.astype(np.float32))


def run_leg(leg, args):
    from muzero_hanoi_amd.muzero import Muzero

    dev = "cpu" if leg == "cpu" else "cuda"
    if leg == "cpu":
        torch.set_num_threads(args.cpu_threads)
    torch.manual_seed(1)
    np.random.seed(1)
    n = args.disks
    mz = Muzero(env=None, s_space_size=3 * n, n_action=6, discount=0.8, dirichlet_alpha=0.25, n_mcts_simulations=25,
                unroll_n_steps=5, batch_s=args.batch, TD_return=True, n_TD_step=10, lr=0.002,
                buffer_size=args.buffer, priority_replay=True, device=dev,
                update_impl={"cpu": "torch", "gpu": "torch", "fused-hostdraw": "fused"}.get(leg, leg),
                device_sampling=False if leg == "fused-hostdraw" else None)
    synthetic_fill(mz, n, args.buffer)
    buf = mz.buffer
    sync = torch.cuda.synchronize if dev == "cuda" else (lambda: None)

    def step():
        s, r, a, p, ret, indx, w = buf.priority_sample(args.batch)
        newp, vl, rl, pl = mz._update(s, r, a, p, ret, w)
        buf.update_priorities(indx, newp)
        return vl

    steps = args.cpu_steps if leg == "cpu" else args.steps
    for _ in range(args.warmup):
        step()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        vl = step()
    sync()
    dt = time.perf_counter() - t0
    # update only (sampling excluded): the same batch over and over
    s, r, a, p, ret, indx, w = buf.priority_sample(args.batch)
    sync()
    t1 = time.perf_counter()
    for _ in range(steps):
        mz._update(s, r, a, p, ret, w)
    sync()
    du = time.perf_counter() - t1
    rec = {"metric": "training_updates_per_sec", "leg": leg, "value": steps / dt, "unit": "updates/s",
           "samples_per_sec": steps * args.batch / dt, "ms_per_update": 1e3 * dt / steps,
           "ms_per_update_no_sampling": 1e3 * du / steps, "steps": steps, "warmup": args.warmup,
           "device_sampling": bool(mz.buffer.device_sampling),
           "final_v_loss": float(vl),
           "config": {"workload": f"hanoi{n}_batch{args.batch}_unroll5_td_prio_buffer{args.buffer}",
                      "device": torch.cuda.get_device_name(0) if dev == "cuda" else "host cpu",
                      "threads": args.cpu_threads if leg == "cpu" else None}}
    print(json.dumps(rec), flush=True)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--legs", default="cpu,gpu,graph,fused,fused-hostdraw")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--cpu-steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--buffer", type=int, default=50000)
    ap.add_argument("--disks", type=int, default=3)
    ap.add_argument("--cpu-threads", type=int, default=1)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    recs = [run_leg(leg, args) for leg in args.legs.split(",")]
    if args.out:
        with open(args.out, "w") as f:
            json.dump(recs, f, indent=1)


if __name__ == "__main__":
    main()
