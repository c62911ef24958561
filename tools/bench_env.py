"""TowersOfHanoi.step throughput (SURVEY.md 6 quotes the reference at ~92k host steps/s):

  reference-host  the reference's step restated in its own form (oracle/py_port.py PortHanoi: tuples, list
                  scans, a NumPy one-hot; env/hanoi.py:47-151, utils.py:9-25), one host core
  drop-in         muzero_hanoi_amd.env.TowersOfHanoi.step: one call = inputs down, one mzh_env_step launch,
                  outputs back (a GPU round trip per step, as the drop-in surface requires a host tuple back)
  batched         HanoiBatch.step: B device-resident envs per mzh_env_step launch, nothing leaves the device

    python tools/bench_env.py [--disks 4] [--seconds 3] [--batch 1048576] [--out profiles/r06_env_bench.json]

Actions are uniform random over the 6 moves (illegal moves included, as a random policy plays), episodes reset
on done.
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


def leg_host(n, seconds):
    from oracle import py_port

    env = py_port.PortHanoi(n, 200)
    env.reset()
    acts = np.random.default_rng(0).integers(0, 6, 1 << 16)
    k, t0 = 0, time.perf_counter()
    while True:
        for _ in range(1000):
            _, _, done, _ = env.step(int(acts[k & 0xFFFF]))
            k += 1
            if done:
                env.reset()
        dt = time.perf_counter() - t0
        if dt > seconds:
            return k, dt


def leg_dropin(n, seconds):
    from muzero_hanoi_amd.env import TowersOfHanoi

    env = TowersOfHanoi(n, 200)
    env.reset()
    acts = np.random.default_rng(0).integers(0, 6, 1 << 16)
    for i in range(50):  # warm-up
        if env.step(int(acts[i]))[2]:
            env.reset()
    k, t0 = 0, time.perf_counter()
    while True:
        for _ in range(200):
            _, _, done, _ = env.step(int(acts[k & 0xFFFF]))
            k += 1
            if done:
                env.reset()
        dt = time.perf_counter() - t0
        if dt > seconds:
            return k, dt


def leg_batched(n, B, steps):
    from muzero_hanoi_amd.env import HanoiBatch

    env = HanoiBatch(n, 200, B)
    env.reset(torch.zeros(B, dtype=torch.int64))
    acts = torch.randint(0, 6, (steps, B), dtype=torch.int32, device=env.device)
    env.step(acts[0])
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for k in range(steps):
        ev[k][0].record()
        env.step(acts[k])
        ev[k][1].record()
        env.active.fill_(1)  # finished episodes continue (a reset without a host round trip)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kern = float(np.median([s.elapsed_time(e) for s, e in ev])) * 1e-3
    return B * steps, dt, kern


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--disks", type=int, default=4)
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    n = a.disks
    rows = []
    k, dt = leg_host(n, a.seconds)
    rows.append({"leg": "reference-host", "steps": k, "seconds": dt, "value": k / dt, "cores": 1})
    k, dt = leg_dropin(n, a.seconds)
    rows.append({"leg": "drop-in", "steps": k, "seconds": dt, "value": k / dt, "us_per_step": dt / k * 1e6})
    k, dt, kern = leg_batched(n, a.batch, 50)
    bytes_per_step = 2 * n + 4 + 3 + 4 + 12 * n  # state read + write, action, flags, counter, obs
    rows.append({"leg": "batched", "envs": a.batch, "steps": k, "seconds": dt, "value": k / dt,
                 "kernel_s_per_launch": kern, "kernel_steps_per_s": a.batch / kern,
                 "kernel_gbps": a.batch * bytes_per_step / kern / 1e9})
    for r in rows:
        r.update(metric="hanoi_env_steps_per_sec", unit="steps/s", disks=n)
        print(json.dumps(r), flush=True)
    if a.out:
        json.dump(rows, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
