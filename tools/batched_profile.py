"""Host-side profile of BatchedSelfPlay.play (4,096 episodes, N=3, S=25, the bench_selfplay batched leg): wall
time per move and cProfile's top entries, to see what the per-move launches and copies cost beside the kernels.

    python tools/batched_profile.py [--episodes 4096]
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
    ap.add_argument("--episodes", type=int, default=4096)
    a = ap.parse_args()
    import numpy as np
    import torch

    from muzero_hanoi_amd.networks import MuZeroNet
    from muzero_hanoi_amd.selfplay import BatchedSelfPlay

    torch.manual_seed(0)
    net = MuZeroNet(9, 6, 0.002, "cuda", TD_return=True)
    sp = BatchedSelfPlay(net, 3, 200, 25)
    starts = np.random.default_rng(2).integers(0, 26, size=a.episodes)
    sp.play(starts[:256], seed=1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = sp.play(starts, seed=2)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    moves = int(res["action"].shape[0])
    print(f"{int(res['steps'].sum())} decisions, {moves} moves in {dt:.3f} s = {dt / moves * 1e3:.3f} ms per move")
    pr = cProfile.Profile()
    pr.enable()
    sp.play(starts, seed=2)
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
