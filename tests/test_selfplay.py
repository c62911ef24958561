"""Self-play driver parity: whole Muzero._play_game episodes of the reference
(tests/golden/episode_*.npz, every network call recorded) replayed through
  * the oracle + the host bookkeeping (CPU), and
  * the drop-in MCTS / TowersOfHanoi on the GPU (play_game with a RecordedNetwork),
must reproduce the reference's trajectory, returns, priorities and RNG position bit for bit.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden
from muzero_hanoi_amd import rng as mrng
from muzero_hanoi_amd import utils as mutils

EPISODES = sorted(f[len("episode_"):-4] for f in os.listdir(GOLDEN) if f.startswith("episode_"))


def _calls(g, t):
    return dict(root_pi=g["out_pi"][t, 0], pi=g["out_pi"][t, 1:], reward=g["out_rwd"][t, 1:].astype(np.float32),
                value=g["out_v"][t, 1:].astype(np.float32))


def _check_episode(g, steps, states, rwds, actions, pi_probs, returns, priorities):
    assert steps == int(g["steps"])
    assert np.array_equal(states, g["states"])
    assert np.array_equal(rwds, g["rwds"]) and np.array_equal(actions, g["actions"])
    assert np.array_equal(pi_probs, g["pi_probs"]) and np.array_equal(returns, g["returns"])
    assert np.array_equal(np.asarray(priorities, np.float32), g["priorities"])
    assert np.array_equal(np.random.random_sample(4), g["post_rng"]), "RNG stream position differs"


@pytest.mark.parametrize("name", EPISODES)
def test_episode_replay_oracle(oracle, name):
    g = golden(f"episode_{name}.npz")
    n, S, det = int(g["n"]), int(g["s"]), bool(g["deterministic"])
    T = mutils.adjust_temperature(int(g["episode"]))
    np.random.seed(int(g["seed"]))
    state = np.zeros(n, np.uint8)  # init_state_idx 0 -> (0,...,0)
    ctr, active = 0, 1
    mm = np.array([[-np.inf, np.inf]])
    ep_state, ep_action, ep_rwd, ep_pi, ep_q = [], [], [], [], []
    obs = np.zeros(3 * n)
    obs[np.arange(n) * 3 + state] = 1
    done = False
    t = 0
    while not done:
        noise, tie, u = mrng.predraw(1, deterministic=det, alpha=0.25)
        c = _calls(g, t)
        o = oracle.search(n, S, obs[None], replay={k: v[None] for k, v in dict(
            root_pi=c["root_pi"], pi=c["pi"], rwd=c["reward"], value=c["value"]).items()},
            noise=noise, tie_idx=tie, action_u=u, temperature=T, deterministic=det, minmax_in=mm)
        assert np.array_equal(o["visits"][0], g["visits"][t])
        mm = np.stack([o["mm_max"], o["mm_min"]], 1)
        a = int(o["action"][0])
        code, state, moved, ctr, active, d, ill = oracle.env_step(state, a, ctr, active, int(g["max_steps"]))
        rwd = {0: 0, 1: 100, -1: -100 / 1000}[code]
        ep_state.append(obs)
        ep_action.append(a)
        ep_rwd.append(rwd)
        ep_pi.append(o["pi"][0])
        ep_q.append(float(o["rootQ"][0]))
        obs = np.zeros(3 * n)
        obs[np.arange(n) * 3 + moved] = 1
        done = bool(d)
        t += 1
    rets = mutils.compute_n_step_returns(ep_rwd, ep_q, int(g["n_td"]), 0.8)
    prio = np.abs(np.array(rets, np.float32) - np.array(ep_q, np.float32))
    out = mutils.organise_transitions(ep_state, ep_rwd, ep_action, ep_pi, rets, 5, 6)
    _check_episode(g, t, *out, prio)


@pytest.mark.gpu
@pytest.mark.parametrize("name", EPISODES)
def test_episode_replay_dropin_gpu(name):
    from muzero_hanoi_amd.env import TowersOfHanoi
    from muzero_hanoi_amd.mcts import MCTS, RecordedNetwork
    from muzero_hanoi_amd.selfplay import play_game

    g = golden(f"episode_{name}.npz")
    n, S = int(g["n"]), int(g["s"])
    net = RecordedNetwork([_calls(g, t) for t in range(int(g["steps"]))], n)
    env = TowersOfHanoi(N=n, max_steps=int(g["max_steps"]))
    mcts = MCTS(discount=0.8, root_dirichlet_alpha=0.25, n_simulations=S, batch_s=256, device="cpu")
    np.random.seed(int(g["seed"]))
    out = play_game(env, mcts, net, int(g["episode"]), bool(g["deterministic"]), discount=0.8, TD_return=True,
                    n_step=int(g["n_td"]), unroll_n_steps=5, n_action=6)
    _check_episode(g, *out)
    assert mcts.min_max_stats.maximum == g["mm"][-1, 0] and mcts.min_max_stats.minimum == g["mm"][-1, 1]


@pytest.mark.gpu
def test_batched_selfplay_vs_oracle(oracle):
    """B envs in lockstep on the GPU == the same episodes simulated with the oracle (MLP mode), each
    env one agent whose MinMaxStats is carried from decision to decision (MCTS/mcts.py:23)."""
    from muzero_hanoi_amd.networks import MuZeroNet
    from muzero_hanoi_amd.selfplay import BatchedSelfPlay

    n, S, B, max_steps, seed = 3, 12, 48, 15, 5
    torch.manual_seed(0)
    net = MuZeroNet(3 * n, 6, 0.002, "cpu", TD_return=True)
    from muzero_hanoi_amd.engine import flat_weights

    flat = flat_weights(net.state_dict())
    starts = np.random.RandomState(1).randint(0, 3 ** n - 1, B)
    mm0 = np.stack([np.linspace(-2.0, 0.0, B), np.linspace(0.5, 3.0, B)], 1)  # agents with history
    mm0[::3] = (-np.inf, np.inf)  # and fresh ones
    res = BatchedSelfPlay(net, n, max_steps, S).play(starts, temperature=1.0, deterministic=False, seed=seed,
                                                     minmax=mm0)
    act = res["action"].cpu().numpy()
    steps = res["steps"].cpu().numpy()
    mm = mm0.copy()
    # oracle simulation with the same per-step draws
    gen = np.random.default_rng(seed)
    st = np.stack([(starts // 3 ** (n - 1 - d)) % 3 for d in range(n)], 1).astype(np.uint8)
    ctr = np.zeros(B, int)
    alive = np.ones(B, bool)
    obs = np.zeros((B, 3 * n), np.float32)
    obs[np.arange(B)[:, None], np.arange(n) * 3 + st] = 1
    t = 0
    while alive.any():
        idx = np.nonzero(alive)[0]
        noise, tie, u = mrng.synthetic_draws(len(idx), deterministic=False, alpha=0.25, seed=int(gen.integers(2**31)))
        o = oracle.search(n, S, obs[idx], flat=flat, support=33, noise=noise, tie_idx=tie, action_u=u, temperature=1.0,
                          minmax_in=mm[idx])
        assert np.array_equal(o["action"], act[t, idx]), f"step {t}"
        mm[idx] = np.stack([o["mm_max"], o["mm_min"]], 1)
        for j, b in enumerate(idx):
            code, s2, moved, c2, a2, d, ill = oracle.env_step(st[b], int(o["action"][j]), int(ctr[b]), 1, max_steps)
            st[b], ctr[b] = s2, c2
            obs[b] = 0
            obs[b, np.arange(n) * 3 + moved] = 1
            if d:
                alive[b] = False
        t += 1
    assert t == act.shape[0]
    assert np.all(steps == (act >= 0).sum(0))
    assert np.array_equal(res["minmax"].cpu().numpy(), mm)


def _fresh_net(n, seed=0):
    from muzero_hanoi_amd.networks import MuZeroNet

    torch.manual_seed(seed)
    return MuZeroNet(3 * n, 6, 0.002, "cpu", TD_return=True)


@pytest.mark.gpu
def test_batched_b1_equals_play_game():
    """One env through BatchedSelfPlay (global NumPy stream, the agent's MinMaxStats carried in and
    out) + episode_records == Muzero._play_game through the drop-ins, bit for bit, RNG included."""
    from muzero_hanoi_amd.env import TowersOfHanoi
    from muzero_hanoi_amd.mcts import MCTS
    from muzero_hanoi_amd.selfplay import BatchedSelfPlay, episode_records, play_game

    n, S, max_steps = 3, 10, 40
    net = _fresh_net(n)
    env = TowersOfHanoi(N=n, max_steps=max_steps, init_state_idx=4)
    mcts = MCTS(discount=0.8, root_dirichlet_alpha=0.25, n_simulations=S, batch_s=256, device="cpu")
    mcts.min_max_stats.maximum, mcts.min_max_stats.minimum = 0.25, -0.5
    np.random.seed(123)
    ref = play_game(env, mcts, net, episode=600, deterministic=False, n_step=10)
    ref_rng = np.random.random_sample(3)
    np.random.seed(123)
    res = BatchedSelfPlay(net, n, max_steps, S).play([4], temperature=0.5, legacy_rng=True, minmax=[[0.25, -0.5]],
                                                     record_obs=True)
    got = episode_records(res, n_step=10)[0]
    assert got[0] == ref[0]
    for a, b in zip(got[1:], ref[1:]):
        assert np.array_equal(np.asarray(a), np.asarray(b))
    assert np.array_equal(np.random.random_sample(3), ref_rng)
    assert tuple(res["minmax"][0].tolist()) == (mcts.min_max_stats.maximum, mcts.min_max_stats.minimum)


@pytest.mark.gpu
@pytest.mark.parametrize("deterministic", [False, True])
def test_play_game_pipelined_and_chained_equal_separate_calls(monkeypatch, deterministic):
    """play_game pipelines the decisions on the device (MCTS.play_episode: decision k+1 launched from decision k's
    device outputs before the host waits for k; the speculative decision after the last one discarded, the
    NumPy stream put back) or chains each run_mcts with its env.step (MCTS.run_mcts_step): the same episodes,
    MinMaxStats, latent actions, env state and NumPy stream as the separate calls -- over several episodes,
    including max_steps endings."""
    from muzero_hanoi_amd.env import TowersOfHanoi
    from muzero_hanoi_amd.mcts import MCTS
    from muzero_hanoi_amd.selfplay import play_game

    n, S, max_steps = 3, 25, 30
    net = _fresh_net(n, seed=3)
    outs = []
    for mode in ("pipelined", "chained", "separate"):
        if mode != "pipelined":
            monkeypatch.setattr(MCTS, "play_episode", lambda *a, **k: None)
        if mode == "separate":
            monkeypatch.setattr(MCTS, "run_mcts_step", lambda *a, **k: None)
        env = TowersOfHanoi(N=n, max_steps=max_steps, init_state_idx=2)
        mcts = MCTS(discount=0.8, root_dirichlet_alpha=0.25, n_simulations=S, batch_s=256, device="cpu")
        np.random.seed(77)
        res = [play_game(env, mcts, net, episode=e, deterministic=deterministic, n_step=10)
               for e in (100, 900, 1500, 2500)]
        outs.append((res, np.random.random_sample(3), mcts.min_max_stats.maximum, mcts.min_max_stats.minimum,
                     [int(t) for t in mcts.return_latent_actions()], env.c_state, env.step_counter, env.reset_check))
    ref = outs[-1]
    for got in outs[:-1]:
        for ea, eb in zip(got[0], ref[0]):
            assert ea[0] == eb[0]
            for x, y in zip(ea[1:], eb[1:]):
                assert np.array_equal(np.asarray(x), np.asarray(y))
        assert np.array_equal(got[1], ref[1]) and got[2:] == ref[2:]


@pytest.mark.gpu
def test_muzero_batched_selfplay():
    """Muzero(selfplay="batched"): a loop's episodes in one lockstep batch.  With one episode per loop
    the buffer, the MCTS instance's MinMaxStats and the RNG stream equal the sequential agent's;
    with several, every episode is recorded with the reference's bookkeeping."""
    from muzero_hanoi_amd.env import TowersOfHanoi
    from muzero_hanoi_amd.muzero import Muzero

    def agent(mode, n_ep):
        torch.manual_seed(3)
        env = TowersOfHanoi(N=3, max_steps=60)
        return Muzero(env=env, s_space_size=9, n_action=6, discount=0.8, dirichlet_alpha=0.25, n_mcts_simulations=8,
                      unroll_n_steps=5, batch_s=16, TD_return=True, n_TD_step=10, lr=0.002, buffer_size=5000,
                      priority_replay=True, device="cuda", n_ep_x_loop=n_ep, selfplay=mode)

    outs = []
    for mode in ("sequential", "batched"):
        mz = agent(mode, 1)
        np.random.seed(9)
        mz.training_loop(n_loops=4, min_replay_size=10**9, print_acc=1000)
        outs.append((len(mz.buffer), mz.buffer.priorities[:len(mz.buffer)].copy(), mz.mcts.min_max_stats.maximum,
                     mz.mcts.min_max_stats.minimum, np.random.random_sample(2)))
    assert outs[0][0] == outs[1][0]
    assert np.array_equal(outs[0][1], outs[1][1])
    assert outs[0][2:4] == outs[1][2:4] and np.array_equal(outs[0][4], outs[1][4])
    mz = agent("batched", 4)
    np.random.seed(9)
    eps = mz._play_games(4, episode=1)
    assert len(eps) == 4
    for steps, states, rwds, actions, pi_probs, returns, prio in eps:
        assert states.shape == (steps, 9) and rwds.shape == (steps, 5) and returns.shape == (steps, 5)
        assert prio.shape == (steps,) and np.allclose(pi_probs.sum(-1), 1.0)
        assert np.all(states.sum(1) == 3)  # one-hot 3-disk observations
