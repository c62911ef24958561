"""Host-side profile of the sequential drop-in self-play loop (selfplay.play_game: MCTS.run_mcts + env.step per
decision, N=3, S=25, as Muzero._play_game runs it): cProfile over ~3 s of episodes, the top entries by own time.

    python tools/dropin_profile.py [--seconds 3]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=3.0)
    a = ap.parse_args()
    import numpy as np
    import torch

    from muzero_hanoi_amd.env import TowersOfHanoi
    from muzero_hanoi_amd.mcts import MCTS
    from muzero_hanoi_amd.networks import MuZeroNet
    from muzero_hanoi_amd.selfplay import play_game

    torch.manual_seed(0)
    net = MuZeroNet(9, 6, 0.002, "cuda", TD_return=True)
    env = TowersOfHanoi(N=3, max_steps=200)
    mcts = MCTS(discount=0.8, root_dirichlet_alpha=0.25, n_simulations=25, batch_s=256, device="cuda")
    np.random.seed(3)
    play_game(env, mcts, net, 1, temperature=1.0)
    pr = cProfile.Profile()
    moves, t0 = 0, time.perf_counter()
    pr.enable()
    while time.perf_counter() - t0 < a.seconds:
        moves += play_game(env, mcts, net, 1, temperature=1.0)[0]
    pr.disable()
    dt = time.perf_counter() - t0
    print(f"{moves} decisions in {dt:.2f} s = {moves / dt:.0f} decisions/s (under cProfile)")
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
