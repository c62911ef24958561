"""Self-play / acting drivers on top of the search.

play_game         Muzero._play_game (Muzero.py:153-207) for one env through the drop-ins: the
                  reference's control flow, RNG consumption and episode bookkeeping, every search
                  and every env step on the GPU.
BatchedSelfPlay   B envs resident on the GPU (HanoiBatch) stepping with search-chosen actions:
                  one mzh_search launch + one mzh_env_step launch per step for all unfinished
                  envs, trajectories kept as device tensors.
evaluate          acting_ablations.get_results (acting_experiments/acting_ablations.py:72-128):
                  episodes from given starts over a range of simulation budgets, error =
                  steps - hanoi_solver(start) (device solver), plus illegal-move rates.
"""
import numpy as np
import torch

from . import rng as _rng
from .engine import hanoi_solver_batch
from .env import HanoiBatch
from .networks import engine_for
from .utils import adjust_temperature, compute_MCreturns, compute_n_step_returns, organise_transitions


def play_game(env, mcts, network, episode, deterministic=False, *, discount=0.8, TD_return=True, n_step=10,
              unroll_n_steps=5, n_action=6, temperature=None):
    """Muzero._play_game: returns (steps, states, rwds, actions, pi_probs, returns, priorities)."""
    episode_state, episode_action, episode_rwd, episode_piProb, episode_rootQ = [], [], [], [], []
    c_state = env.reset()
    done = False
    step = 0
    T = adjust_temperature(episode) if temperature is None else temperature
    while not done:
        action, pi_prob, rootQ = mcts.run_mcts(c_state, network, temperature=T, deterministic=deterministic)
        n_state, rwd, done, _ = env.step(action)
        step += 1
        episode_state.append(c_state)
        episode_action.append(action)
        episode_rwd.append(rwd)
        episode_piProb.append(pi_prob)
        episode_rootQ.append(rootQ)
        c_state = n_state
    if TD_return:
        episode_returns = compute_n_step_returns(episode_rwd, episode_rootQ, n_step, discount)
    else:
        episode_returns = compute_MCreturns(episode_rwd, discount)
    priorities = np.abs(np.array(episode_returns, dtype=np.float32) - np.array(episode_rootQ, dtype=np.float32))
    states, rwds, actions, pi_probs, returns = organise_transitions(
        episode_state, episode_rwd, episode_action, episode_piProb, episode_returns, unroll_n_steps, n_action)
    return step, states, rwds, actions, pi_probs, returns, priorities


class BatchedSelfPlay:
    """B independent episodes in lockstep on one GPU.  Each root of a step is an independent
    search (its own MinMaxStats), i.e. the semantics of a fresh MCTS per decision; with
    `legacy_rng` the draws come from NumPy's global stream (B = 1 reproduces play_game's draws),
    otherwise from a vectorised Generator(seed)."""

    def __init__(self, network, n_disks, max_steps, n_simulations, *, discount=0.8, dirichlet_alpha=0.25,
                 root_exploration_eps=0.25, goal_peg=2):
        self.network = network
        self.N, self.max_steps, self.S = n_disks, max_steps, n_simulations
        self.discount, self.alpha, self.eps, self.goal_peg = discount, dirichlet_alpha, root_exploration_eps, goal_peg

    def play(self, start_idx, temperature=1.0, deterministic=False, seed=0, legacy_rng=False):
        start = torch.as_tensor(np.asarray(start_idx), dtype=torch.int64)
        B = int(start.shape[0])
        eng = engine_for(self.network, self.S, B)
        dev = eng.device
        env = HanoiBatch(self.N, self.max_steps, B, goal_peg=self.goal_peg, device=dev)
        obs = env.reset(start.to(dev))
        gen = np.random.default_rng(seed)
        active = torch.ones(B, dtype=torch.bool, device=dev)
        steps = torch.zeros(B, dtype=torch.int32, device=dev)
        illegal_n = torch.zeros(B, dtype=torch.int32, device=dev)
        rec = dict(action=[], reward=[], pi=[], root_q=[], active=[])
        while True:
            idx = active.nonzero().squeeze(1)
            n = int(idx.numel())
            if n == 0:
                break
            if legacy_rng:
                noise, tie, u = _rng.predraw(n, deterministic=deterministic, alpha=self.alpha, eps=self.eps)
            else:
                noise, tie, u = _rng.synthetic_draws(n, deterministic=deterministic, alpha=self.alpha, eps=self.eps,
                                                     seed=int(gen.integers(2**31)))
            t = lambda a: None if a is None else torch.as_tensor(a).to(dev)
            out = eng.search(self.S, obs=obs.index_select(0, idx), tie_idx=t(tie), noise=t(noise), action_u=t(u),
                             temperature=float(temperature), deterministic=bool(deterministic),
                             discount=self.discount, eps=self.eps)
            # step only the unfinished envs (gather -> one env kernel -> scatter)
            sub_state = env.state.index_select(0, idx).contiguous()
            sub_ctr = env.step_ctr.index_select(0, idx).contiguous()
            sub_act = env.active.index_select(0, idx).contiguous()
            from .engine import env_step

            sub_obs = torch.empty((n, 3 * self.N), dtype=torch.float32, device=dev)
            code, done, ill = env_step(self.N, self.max_steps, sub_state, out["action"], sub_ctr, sub_act,
                                       goal_peg=self.goal_peg, obs=sub_obs, err=env.err)
            env.state.index_copy_(0, idx, sub_state)
            env.step_ctr.index_copy_(0, idx, sub_ctr)
            env.active.index_copy_(0, idx, sub_act)
            obs = obs.index_copy(0, idx, sub_obs)
            steps.index_add_(0, idx, torch.ones_like(idx, dtype=torch.int32))
            illegal_n.index_add_(0, idx, ill.to(torch.int32))
            full = lambda v, fill, dt: torch.full((B,) + tuple(v.shape[1:]), fill, dtype=dt, device=dev).index_copy(0, idx, v.to(dt))
            rec["action"].append(full(out["action"], -1, torch.int32))
            rec["reward"].append(full(HanoiBatch.reward_value(code), 0.0, torch.float64))
            rec["pi"].append(full(out["pi"], 0.0, torch.float64))
            rec["root_q"].append(full(out["root_q"], 0.0, torch.float64))
            rec["active"].append(active.clone())
            active = active.index_copy(0, idx, done == 0)
        res = {k: torch.stack(v) if v else torch.empty(0, device=dev) for k, v in rec.items()}
        res["steps"] = steps
        res["illegal"] = illegal_n
        res["start_idx"] = start.to(dev)
        return res


def evaluate(network, n_disks, start_idx, n_sims_range, *, max_steps=200, temperature=1.0, seed=0,
             goal_peg=2, deterministic=False):
    """acting_ablations.get_results over a batch of starts: mean (steps - optimal) per budget,
    plus the illegal-move rate (illegal_move_rate_comparison.py:27-50)."""
    start = torch.as_tensor(np.asarray(start_idx), dtype=torch.int64)
    data = []
    for n in n_sims_range:
        sp = BatchedSelfPlay(network, n_disks, max_steps, int(n), goal_peg=goal_peg)
        res = sp.play(start, temperature=temperature, deterministic=deterministic, seed=seed)
        dev = res["steps"].device
        pw = 3 ** torch.arange(n_disks - 1, -1, -1, device=dev)
        st = ((start.to(dev)[:, None] // pw) % 3).to(torch.uint8)
        opt = hanoi_solver_batch(n_disks, st, goal_peg)
        err = (res["steps"] - opt).double()
        ill = res["illegal"].double().sum() / res["steps"].double().sum()
        data.append([int(n), float(err.mean()), float(ill)])
    return data
