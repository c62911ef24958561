"""Self-play / acting drivers on top of the search.

play_game          Muzero._play_game (Muzero.py:153-207) for one env through the drop-ins: the
                   reference's control flow, RNG consumption and episode bookkeeping, every search
                   and every env step on the GPU.
BatchedSelfPlay    B envs resident on the GPU (HanoiBatch) stepping with search-chosen actions:
                   one mzh_search launch + one mzh_env_step launch per step for all unfinished
                   envs.  Each env is one agent with its own MCTS instance: its MinMaxStats
                   (MCTS/mcts.py:23, never reset) is carried from decision to decision
                   (minmax_out -> minmax_in), starting from the `minmax` handed in.
episode_records    the reference's per-episode bookkeeping (returns, priorities,
                   organise_transitions) of every env of a BatchedSelfPlay run.
evaluate           acting_ablations.get_results (acting_experiments/acting_ablations.py:72-128)
                   and illegal_move_rate (illegal_move_rate_comparison.py:27-50) over episodes:
                   error = steps - hanoi_solver(start), per-episode illegal-move rates (mean and
                   standard error).  sequential=True is the reference's own schedule -- one MCTS
                   instance, episodes one after another, the global NumPy stream -- and reproduces
                   get_results exactly; otherwise a budget's episodes run as one batch, each with
                   its own persistent MinMaxStats.

RNG: with legacy_rng the draws come from NumPy's global stream (rng.predraw) in the order the
reference consumes them when one env plays at a time (B = 1, or sequential=True); a batch of
B > 1 lockstep envs draws, per step, for its unfinished envs in env order -- a different
interleaving than B sequential episodes, so only the B = 1 forms are stream-identical.
"""
import numpy as np
import torch

from . import rng as _rng
from .engine import env_step as _env_step
from .engine import hanoi_solver_batch
from .env import HanoiBatch
from .networks import engine_for
from .utils import adjust_temperature, compute_MCreturns, compute_n_step_returns, organise_transitions

# acting_experiments/acting_ablations.py:49-68: the named 3-disk starts (distance to goal 7 / 3 / 1)
START_STATES = {"ES": (2, 2, 0), "MS": (0, 0, 2), "LS": (1, 2, 2)}


def state_index(state):
    """reference state tuple -> index into TowersOfHanoi.states (itertools.product order)"""
    idx = 0
    for s in state:
        idx = idx * 3 + int(s)
    return idx


def index_state(idx, n_disks):
    return tuple(int(idx // 3 ** (n_disks - 1 - d)) % 3 for d in range(n_disks))


def play_game(env, mcts, network, episode, deterministic=False, *, discount=0.8, TD_return=True, n_step=10,
              unroll_n_steps=5, n_action=6, temperature=None):
    """Muzero._play_game: returns (steps, states, rwds, actions, pi_probs, returns, priorities)."""
    episode_state, episode_action, episode_rwd, episode_piProb, episode_rootQ = [], [], [], [], []
    c_state = env.reset()
    done = False
    step = 0
    T = adjust_temperature(episode) if temperature is None else temperature
    # our MCTS + TowersOfHanoi: the decisions pipelined on the device (MCTS.play_episode), else the search and
    # the env step as chained launches with one synchronisation per decision (MCTS.run_mcts_step)
    ours = hasattr(env, "_launch_step")
    pipe = getattr(mcts, "play_episode", None) if ours else None
    r = pipe(env, network, T, deterministic) if pipe is not None and c_state is env.oneH_c_state else None
    if r is not None:
        step, episode_state, episode_action, episode_rwd, episode_piProb, episode_rootQ = r
        done = True
    chain = getattr(mcts, "run_mcts_step", None) if ours else None
    while not done:
        r = chain(c_state, network, T, deterministic, env) if chain is not None else None
        if r is not None:
            action, pi_prob, rootQ, (n_state, rwd, done, _) = r
        else:
            action, pi_prob, rootQ = mcts.run_mcts(c_state, network, temperature=T, deterministic=deterministic)
            n_state, rwd, done, _ = env.step(action)
        step += 1
        episode_state.append(c_state)
        episode_action.append(action)
        episode_rwd.append(rwd)
        episode_piProb.append(pi_prob)
        episode_rootQ.append(rootQ)
        c_state = n_state
    returns, priorities, trans = _bookkeeping(episode_state, episode_rwd, episode_action, episode_piProb,
                                              episode_rootQ, discount=discount, TD_return=TD_return, n_step=n_step,
                                              unroll_n_steps=unroll_n_steps, n_action=n_action)
    states, rwds, actions, pi_probs, returns = trans
    return step, states, rwds, actions, pi_probs, returns, priorities


def _bookkeeping(episode_state, episode_rwd, episode_action, episode_piProb, episode_rootQ, *, discount, TD_return,
                 n_step, unroll_n_steps, n_action):
    """Muzero.py:188-205: returns (n-step TD or Monte Carlo), priorities |return - root Q| in fp32,
    and the unroll targets (organise_transitions draws one np.random.randint)."""
    if TD_return:
        episode_returns = compute_n_step_returns(episode_rwd, episode_rootQ, n_step, discount)
    else:
        episode_returns = compute_MCreturns(episode_rwd, discount)
    priorities = np.abs(np.array(episode_returns, dtype=np.float32) - np.array(episode_rootQ, dtype=np.float32))
    trans = organise_transitions(episode_state, episode_rwd, episode_action, episode_piProb, episode_returns,
                                 unroll_n_steps, n_action)
    return episode_returns, priorities, trans


class BatchedSelfPlay:
    """B independent agents in lockstep on one GPU, one MCTS instance (MinMaxStats) each."""

    def __init__(self, network, n_disks, max_steps, n_simulations, *, discount=0.8, dirichlet_alpha=0.25,
                 root_exploration_eps=0.25, goal_peg=2, np1_ucb=False):
        self.network = network
        self.N, self.max_steps, self.S = n_disks, max_steps, n_simulations
        self.discount, self.alpha, self.eps, self.goal_peg = discount, dirichlet_alpha, root_exploration_eps, goal_peg
        self.np1_ucb = np1_ucb

    def _engine(self, B):
        from .mcts import RecordedNetwork, _replay_engine

        if isinstance(self.network, RecordedNetwork):
            if B != 1:
                raise ValueError("a RecordedNetwork replays one sequential stream of searches: B must be 1")
            return _replay_engine(self.N, self.S), True
        return engine_for(self.network, self.S, B), False

    def play(self, start_idx, temperature=1.0, deterministic=False, seed=0, legacy_rng=False, minmax=None,
             record_obs=False):
        """Play every env from start_idx[b] until done (goal or max_steps).

        minmax: [B, 2] (maximum, minimum) of each agent's MinMaxStats at the start (default: fresh,
        -inf / +inf); the final values come back as res["minmax"].  Returns device tensors:
        per step t (rows of envs that were still playing): action, reward, pi, root_q, active,
        obs (record_obs); per env: steps, illegal (count), start_idx, minmax."""
        start = torch.as_tensor(np.asarray(start_idx), dtype=torch.int64).reshape(-1)
        B = int(start.shape[0])
        eng, replay = self._engine(B)
        dev = eng.device
        env = HanoiBatch(self.N, self.max_steps, B, goal_peg=self.goal_peg, device=dev)
        obs = env.reset(start.to(dev))
        gen = np.random.default_rng(seed)
        mm = torch.empty((B, 2), dtype=torch.float64, device=dev)
        if minmax is None:
            mm[:, 0], mm[:, 1] = -float("inf"), float("inf")
        else:
            mm.copy_(torch.as_tensor(np.asarray(minmax, np.float64)).reshape(B, 2))
        active = torch.ones(B, dtype=torch.bool, device=dev)
        steps = torch.zeros(B, dtype=torch.int32, device=dev)
        illegal_n = torch.zeros(B, dtype=torch.int32, device=dev)
        rec = dict(action=[], reward=[], pi=[], root_q=[], active=[])
        if record_obs:
            rec["obs"] = []
        t = lambda a: None if a is None else torch.as_tensor(a).to(dev)
        cut = lambda a, m: None if a is None else a[:m]
        # synthetic draws: a move's batch is drawn on the host while the GPU still runs the previous move, for
        # that move's count of envs (an upper bound), and cut to the count left once it is known (the draws
        # of n envs are the first n rows of a larger draw, rng.synthetic_draws)
        pre = None
        while True:
            idx = active.nonzero().squeeze(1)
            n = int(idx.numel())
            if n == 0:
                break
            if legacy_rng:
                noise, tie, u = _rng.predraw(n, deterministic=deterministic, alpha=self.alpha, eps=self.eps)
            else:
                if pre is None:
                    pre = _rng.synthetic_draws(n, deterministic=deterministic, alpha=self.alpha, eps=self.eps,
                                               seed=int(gen.integers(2**31)))
                noise, tie, u = (cut(x, n) for x in pre)
                pre = None
            rp = None
            if replay:
                call = self.network.next_call()
                rp = {k: torch.as_tensor(np.asarray(call[k], np.float32)).to(dev)[None]
                      for k in ("root_pi", "pi", "reward", "value")}
            sub_obs_in = obs.index_select(0, idx)
            out = eng.search(self.S, obs=None if replay else sub_obs_in, replay=rp, tie_idx=t(tie), noise=t(noise),
                             action_u=t(u), minmax_in=mm.index_select(0, idx), temperature=float(temperature),
                             deterministic=bool(deterministic), discount=self.discount, eps=self.eps,
                             np1_ucb=self.np1_ucb)
            mm.index_copy_(0, idx, out["minmax"])
            # step only the unfinished envs (gather -> one env kernel -> scatter)
            sub_state = env.state.index_select(0, idx).contiguous()
            sub_ctr = env.step_ctr.index_select(0, idx).contiguous()
            sub_act = env.active.index_select(0, idx).contiguous()
            sub_obs = torch.empty((n, 3 * self.N), dtype=torch.float32, device=dev)
            code, done, ill = _env_step(self.N, self.max_steps, sub_state, out["action"], sub_ctr, sub_act,
                                        goal_peg=self.goal_peg, obs=sub_obs, err=env.err)
            env.state.index_copy_(0, idx, sub_state)
            env.step_ctr.index_copy_(0, idx, sub_ctr)
            env.active.index_copy_(0, idx, sub_act)
            steps.index_add_(0, idx, torch.ones_like(idx, dtype=torch.int32))
            illegal_n.index_add_(0, idx, ill.to(torch.int32))
            full = lambda v, fill, dt: torch.full((B,) + tuple(v.shape[1:]), fill, dtype=dt, device=dev).index_copy(
                0, idx, v.to(dt))
            rec["action"].append(full(out["action"], -1, torch.int32))
            rec["reward"].append(full(HanoiBatch.reward_value(code), 0.0, torch.float64))
            rec["pi"].append(full(out["pi"], 0.0, torch.float64))
            rec["root_q"].append(full(out["root_q"], 0.0, torch.float64))
            rec["active"].append(active.clone())
            if record_obs:
                rec["obs"].append(full(sub_obs_in, 0.0, torch.float32))
            obs = obs.index_copy(0, idx, sub_obs)
            active = active.index_copy(0, idx, done == 0)
            if not legacy_rng and not replay:  # the next move's draws, overlapping this move's kernels
                pre = _rng.synthetic_draws(n, deterministic=deterministic, alpha=self.alpha, eps=self.eps,
                                           seed=int(gen.integers(2**31)))
        res = {k: torch.stack(v) if v else torch.empty(0, device=dev) for k, v in rec.items()}
        res["steps"] = steps
        res["illegal"] = illegal_n
        res["start_idx"] = start.to(dev)
        res["minmax"] = mm
        return res


def episode_records(res, *, discount=0.8, TD_return=True, n_step=10, unroll_n_steps=5, n_action=6):
    """Muzero._play_game's return value for every env of a BatchedSelfPlay.play(record_obs=True)
    result, in env order: (steps, states, rwds, actions, pi_probs, returns, priorities)."""
    host = {k: res[k].cpu().numpy() for k in ("action", "reward", "pi", "root_q", "active", "obs", "steps")}
    out = []
    for b in range(host["steps"].shape[0]):
        T = int(host["steps"][b])
        states = [host["obs"][t, b].astype(np.float64) for t in range(T)]
        rwds = [_reward_py(host["reward"][t, b]) for t in range(T)]
        actions = [int(host["action"][t, b]) for t in range(T)]
        pis = [host["pi"][t, b] for t in range(T)]
        rootq = [float(host["root_q"][t, b]) for t in range(T)]
        _, priorities, trans = _bookkeeping(states, rwds, actions, pis, rootq, discount=discount, TD_return=TD_return,
                                            n_step=n_step, unroll_n_steps=unroll_n_steps, n_action=n_action)
        out.append((T,) + tuple(trans[:4]) + (trans[4], priorities))
    return out


def _reward_py(r):
    """the reference's Python reward objects (env/hanoi.py:60-72: int 0 / 100 or float -0.1)"""
    r = float(r)
    return 0 if r == 0.0 else (100 if r == 100.0 else r)


# ------------------------------------------------------------------------------------------------
# evaluation (acting_ablations.get_results, illegal_move_rate_comparison.illegal_move_rate)
# ------------------------------------------------------------------------------------------------
def _start_index(start, n_disks):
    if start in START_STATES:
        if n_disks != 3:
            raise ValueError("the ES / MS / LS starts are 3-disk states (acting_ablations.py:49-68)")
        return state_index(START_STATES[start])
    return int(start)


def _random_start(n_disks, goal_peg):
    """TowersOfHanoi.random_reset's draw loop (env/hanoi.py:103-109) on the global NumPy stream"""
    goal = state_index((goal_peg,) * n_disks)
    while True:
        i = np.random.randint(3 ** n_disks)
        if i != goal:
            return i


def evaluate(network, n_disks, n_sims_range, *, episodes=1, start=None, start_idx=None, max_steps=200,
             temperature=1.0, deterministic=False, sequential=False, legacy_rng=None, seed=0, goal_peg=2, minmax=None,
             np1_ucb=False):
    """Episodes per simulation budget, scored like the reference's acting scripts.

    start: None -> random_reset starts (env/hanoi.py:103-109); "ES" / "MS" / "LS" or a state index
    -> that fixed start (acting_ablations.py:49-68); start_idx: explicit per-episode start indices.
    sequential: one MCTS instance for every episode and budget (its MinMaxStats carried across all
    of them, `minmax` its initial value), episodes one after another, draws (random starts
    included) from the global NumPy stream -- get_results' schedule.  Otherwise each budget's
    episodes run as one batch, each episode its own agent with a fresh MinMaxStats.
    Returns dict(data=[[n, mean error]] (get_results' value), illegal=[[n, mean rate, std error]]
    (illegal_move_rate's value per budget), errors / steps / illegal_rates per budget, minmax).
    minmax (in and out) is the carried chain of the sequential schedule only: with
    sequential=False every agent starts fresh, `minmax` must be None and None is returned."""
    if not sequential and minmax is not None:
        raise ValueError("evaluate: minmax applies to the sequential schedule only (batched agents start fresh)")
    legacy_rng = sequential if legacy_rng is None else legacy_rng
    data, illegal, errors_all, steps_all, rates_all = [], [], [], [], []
    mm = None if minmax is None else np.asarray(minmax, np.float64).reshape(1, 2)
    for n in n_sims_range:
        sp = BatchedSelfPlay(network, n_disks, max_steps, int(n), goal_peg=goal_peg, np1_ucb=np1_ucb)
        if sequential:
            steps, ill, starts = [], [], []
            for ep in range(episodes):
                if start_idx is not None:
                    s0 = int(np.asarray(start_idx).reshape(-1)[ep])
                elif start is None:
                    s0 = _random_start(n_disks, goal_peg)
                else:
                    s0 = _start_index(start, n_disks)
                res = sp.play([s0], temperature=temperature, deterministic=deterministic, legacy_rng=legacy_rng,
                              minmax=mm, seed=seed + ep)
                mm = res["minmax"].cpu().numpy()
                steps.append(int(res["steps"][0]))
                ill.append(int(res["illegal"][0]))
                starts.append(s0)
            steps, ill, starts = np.array(steps), np.array(ill), np.array(starts)
        else:
            if start_idx is not None:
                starts = np.asarray(start_idx, np.int64).reshape(-1)
            elif start is None:
                g = np.random.default_rng(seed)
                goal = state_index((goal_peg,) * n_disks)
                starts = g.integers(0, 3 ** n_disks - 1, size=episodes)
                starts = starts + (starts >= goal)  # uniform over the non-goal states
            else:
                starts = np.full(episodes, _start_index(start, n_disks), np.int64)
            res = sp.play(starts, temperature=temperature, deterministic=deterministic, legacy_rng=legacy_rng,
                          seed=seed)
            steps, ill = res["steps"].cpu().numpy(), res["illegal"].cpu().numpy()
        dev = torch.device("cuda", torch.cuda.current_device())
        st = torch.tensor([index_state(int(i), n_disks) for i in starts], dtype=torch.uint8, device=dev)
        opt = hanoi_solver_batch(n_disks, st, goal_peg).cpu().numpy()
        err = steps - opt
        rates = ill / np.maximum(steps, 1)
        data.append([int(n), float(sum(int(e) for e in err) / len(err))])
        sem = float(np.std(rates, ddof=1) / np.sqrt(len(rates))) if len(rates) > 1 else float("nan")
        illegal.append([int(n), float(np.mean(rates)), sem])
        errors_all.append(err)
        steps_all.append(steps)
        rates_all.append(rates)
    return dict(data=data, illegal=illegal, errors=errors_all, steps=steps_all, illegal_rates=rates_all,
                minmax=mm if sequential else None)
