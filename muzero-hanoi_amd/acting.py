"""Acting / evaluation drop-ins: the functions the reference's acting scripts are built from, with
the same signatures, running on the drop-in TowersOfHanoi / MCTS / MuZeroNet (every search one
fused kernel launch, every env step the integer kernel).

  get_starting_state   acting_experiments/acting_ablations.py:49-68 (ES / MS / LS / random)
  ablate_networks      acting_experiments/acting_ablations.py:29-45 (head re-initialisation)
  get_results          acting_experiments/acting_ablations.py:72-128 (error vs the optimal move count
                       per simulation budget; one MCTS instance, MinMaxStats carried throughout)
  illegal_move_rate    illegal_move_rate_comparison.py:27-50 (per-episode rates: mean, std error)

They run one decision at a time, exactly as the reference does (same RNG stream, same MinMaxStats
chain); selfplay.evaluate is the batched form (sequential=True reproduces get_results).
"""
import logging

import numpy as np
import torch

from .checkpoint import ablate_networks  # noqa: F401  (acting_ablations.py:29-45; one implementation)
from .hanoi_utils import hanoi_solver
from .selfplay import START_STATES

_LABELS = {0: "ES", 1: "MS", 2: "LS"}


def get_starting_state(env, start=None):
    """Point env.init_state_idx at the named start (0 = ES, 1 = MS, 2 = LS; 3-disk states chosen
    off the training trajectory) and return its file label; None leaves the env for random_reset."""
    if start is None:
        return "RandState"
    label = _LABELS[start]
    env.init_state_idx = env.states.index(START_STATES[label])
    return label


def _episode(env, start, networks, mcts, temperature, deterministic=False):
    """one episode: reset (fixed or random start), search + step until done; returns
    (start state, steps, illegal moves)"""
    c_state = env.reset() if start else env.random_reset()
    s0 = tuple(env.current_state())
    steps = illegal = 0
    done = False
    while not done:
        action, _, _ = mcts.run_mcts(c_state, networks, temperature=temperature, deterministic=deterministic)
        c_state, _, done, illegal_move = env.step(action)
        steps += 1
        illegal += int(illegal_move)
    return s0, steps, illegal


@torch.no_grad()
def get_results(env, start, networks, mcts, episode, n_mcts_simulations_range, temperature):
    """[[n_simulations, mean(steps - optimal moves)]] over `episode` episodes per budget."""
    data = []
    for n in n_mcts_simulations_range:
        mcts.n_simulations = n
        errors = []
        for _ in range(episode):
            s0, steps, _ = _episode(env, start is not None, networks, mcts, temperature)
            errors.append(steps - hanoi_solver(s0))
        data.append([n, sum(errors) / len(errors)])
    logging.info(data)
    return data


def illegal_move_rate(env, networks, mcts, episodes=100, temperature=0.0, fixed_start=False):
    """(mean, standard error) of the per-episode illegal-move rates (illegal moves / moves)."""
    rates = []
    for _ in range(episodes):
        _, steps, illegal = _episode(env, fixed_start, networks, mcts, temperature)
        if steps > 0:
            rates.append(illegal / steps)
    if not rates:
        return 0.0, 0.0
    return float(np.mean(rates)), float(np.std(rates, ddof=1) / np.sqrt(len(rates)))
