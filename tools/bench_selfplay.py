"""Self-play / acting throughput: decisions per second, one decision = one
MCTS search of S simulations from the current state + one TowersOfHanoi step, episodes from
uniform random non-goal starts until the goal or max_steps (Muzero._play_game, Muzero.py:153-207;
acting_ablations.get_results, acting_experiments/acting_ablations.py:72-128).  Reference training
config: N=3, max_steps=200, S=25, T=1 stochastic, random-init MuZeroNet(TD_return=True).

Legs:
  batched   B episodes in lockstep on one GPU (selfplay.BatchedSelfPlay: one search launch and one
            env-kernel launch per move over every unfinished episode)
  batched-legacy  the same with every draw from NumPy's global legacy stream in the reference's
            order (legacy_rng=True; rng.predraw, the bit-exact mode)
  drop-in   the reference's sequential loop through the drop-ins (selfplay.play_game: one
            MCTS.run_mcts launch and one env.step per decision, as Muzero._play_game runs it)
  cpu       the reference algorithm on one host core (bench.cpu_baseline_selfplay: oracle/py_port.py's
            object-tree MCTS with a batch-1 torch-CPU MLP + the C env restatement), bounded to
            --cpu-seconds

  python tools/bench_selfplay.py [--legs batched,batched-legacy,drop-in,cpu] [--episodes 4096] [--sims 25]
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


def start_states(n_disks, B, seed):
    g = np.random.default_rng(seed)
    return g.integers(0, 3 ** n_disks - 1, size=B)  # every state index but the goal's


def leg_batched(args, net):
    from muzero_hanoi_amd.selfplay import BatchedSelfPlay

    sp = BatchedSelfPlay(net, args.disks, args.max_steps, args.sims)
    sp.play(start_states(args.disks, min(args.episodes, 256), 1), seed=1)  # warm-up (engine, kernels)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = sp.play(start_states(args.disks, args.episodes, 2), seed=2)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    moves = int(res["steps"].sum())
    return dict(decisions=moves, episodes=args.episodes, seconds=dt,
                solved=int((res["steps"] < args.max_steps).sum()))


def leg_batched_legacy(args, net):
    """the batched leg with every draw from NumPy's global legacy stream in the reference's order
    (legacy_rng=True: rng.predraw per move over the unfinished episodes) -- the bit-exact mode"""
    from muzero_hanoi_amd.selfplay import BatchedSelfPlay

    sp = BatchedSelfPlay(net, args.disks, args.max_steps, args.sims)
    np.random.seed(1)
    sp.play(start_states(args.disks, min(args.episodes, 256), 1), legacy_rng=True)  # warm-up
    torch.cuda.synchronize()
    np.random.seed(2)
    t0 = time.perf_counter()
    res = sp.play(start_states(args.disks, args.episodes, 2), legacy_rng=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    moves = int(res["steps"].sum())
    return dict(decisions=moves, episodes=args.episodes, seconds=dt,
                solved=int((res["steps"] < args.max_steps).sum()))


def leg_dropin(args, net):
    from muzero_hanoi_amd.env import TowersOfHanoi
    from muzero_hanoi_amd.mcts import MCTS
    from muzero_hanoi_amd.selfplay import play_game

    env = TowersOfHanoi(N=args.disks, max_steps=args.max_steps)
    mcts = MCTS(discount=0.8, root_dirichlet_alpha=0.25, n_simulations=args.sims, batch_s=256, device="cuda")
    np.random.seed(3)
    play_game(env, mcts, net, 1, temperature=1.0)  # warm-up
    moves, eps_done = 0, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.dropin_seconds:
        env.init_state_idx = int(start_states(args.disks, 1, 100 + eps_done)[0])
        steps = play_game(env, mcts, net, 1, temperature=1.0)[0]
        moves += steps
        eps_done += 1
    dt = time.perf_counter() - t0
    return dict(decisions=moves, episodes=eps_done, seconds=dt)


def leg_cpu(args, net):
    from bench import cpu_baseline_selfplay

    moves, eps_done, dt = cpu_baseline_selfplay(args.disks, args.sims, args.max_steps, args.cpu_seconds,
                                                net.state_dict(),
                                                lambda k: start_states(args.disks, 1, 200 + k)[0])
    return dict(decisions=moves, episodes=eps_done, seconds=dt, cores=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--legs", default="batched,drop-in,cpu")
    ap.add_argument("--episodes", type=int, default=4096)
    ap.add_argument("--disks", type=int, default=3)
    ap.add_argument("--max-steps", type=int, default=200)
    ap.add_argument("--sims", type=int, default=25)
    ap.add_argument("--dropin-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from muzero_hanoi_amd.networks import MuZeroNet

    torch.manual_seed(1)
    recs = []
    for leg in args.legs.split(","):
        dev = "cpu" if leg == "cpu" else "cuda"
        torch.manual_seed(1)
        net = MuZeroNet(3 * args.disks, 6, 0.002, dev, TD_return=True).to(dev)
        r = {"batched": leg_batched, "batched-legacy": leg_batched_legacy, "drop-in": leg_dropin,
             "cpu": leg_cpu}[leg](args, net)
        r.update(leg=leg, metric="selfplay_decisions_per_sec", value=r["decisions"] / r["seconds"],
                 unit="decisions/s", sims_per_sec=r["decisions"] * args.sims / r["seconds"],
                 config={"workload": f"hanoi{args.disks}_s{args.sims}_maxsteps{args.max_steps}",
                         "episodes": r["episodes"], "T": 1.0, "stochastic": True})
        print(json.dumps(r), flush=True)
        recs.append(r)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(recs, f, indent=1)


if __name__ == "__main__":
    main()
