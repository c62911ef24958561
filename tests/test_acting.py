"""Acting / evaluation parity against runs of the reference itself:
tests/golden/acting_*.npz are acting_ablations.get_results runs (acting_experiments/
acting_ablations.py:72-128: one MCTS instance for every budget and episode, ES or random starts),
tests/golden/illegal_*.npz illegal_move_rate_comparison.illegal_move_rate runs (:27-50), each with
every network output recorded (tests/golden/gen_golden.py gen_acting / gen_illegal).

  CPU  the oracle search + oracle env + host bookkeeping replay them: pins the fixtures against
       the restatement (errors, actions, MinMaxStats chain, RNG position);
  GPU  the drop-ins (acting.get_results / acting.illegal_move_rate on the drop-in MCTS and
       TowersOfHanoi) and the batched evaluator in its sequential schedule
       (selfplay.evaluate(sequential=True)) replay them bit for bit.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden
from muzero_hanoi_amd import rng as mrng

ACTING = sorted(f[len("acting_"):-4] for f in os.listdir(GOLDEN) if f.startswith("acting_"))
ILLEGAL = sorted(f[len("illegal_"):-4] for f in os.listdir(GOLDEN) if f.startswith("illegal_"))


def recorded_calls(g):
    """per run_mcts call: the recorded root policy and per-simulation outputs (RecordedNetwork format)"""
    calls, off = [], 0
    for k, S in enumerate(g["run_S"]):
        S = int(S)
        calls.append(dict(root_pi=g["run_root_pi"][k], pi=g["run_pi"][off:off + S],
                          reward=g["run_reward"][off:off + S], value=g["run_value"][off:off + S]))
        off += S
    return calls


def _oracle_episodes(oracle, g, budgets, episodes, fixed_start, init_idx, temperature):
    """the reference's acting loop on the oracle: returns (data, rates, actions, mm chain)"""
    from muzero_hanoi_amd.hanoi_utils import hanoi_solver
    from muzero_hanoi_amd.selfplay import index_state

    n, max_steps = int(g["n"]), int(g["max_steps"])
    calls = recorded_calls(g)
    k = 0
    mm = np.array([[-np.inf, np.inf]])
    data, rates, actions, mms = [], [], [], []
    for S in budgets:
        errors = []
        for _ in range(episodes):
            if fixed_start:
                idx = init_idx
            else:  # env/hanoi.py:103-109 on the global stream
                while True:
                    idx = np.random.randint(3 ** n)
                    if idx != 3 ** n - 1:
                        break
            st = np.array(index_state(idx, n), np.uint8)
            s0 = tuple(int(x) for x in st)
            ctr, active, done, steps, illegal = 0, 1, 0, 0, 0
            while not done:
                obs = np.zeros(3 * n)
                obs[np.arange(n) * 3 + st] = 1
                noise, tie, u = mrng.predraw(1, deterministic=False, alpha=0.25)
                c = calls[k]
                k += 1
                o = oracle.search(n, int(S), obs[None], replay=dict(root_pi=c["root_pi"][None], pi=c["pi"][None],
                                                                     rwd=c["reward"][None], value=c["value"][None]),
                                  noise=noise, tie_idx=tie, action_u=u, temperature=temperature, minmax_in=mm)
                mm = np.stack([o["mm_max"], o["mm_min"]], 1)
                a = int(o["action"][0])
                actions.append(a)
                mms.append(mm[0].copy())
                _, st, _, ctr, active, done, ill = oracle.env_step(st, a, ctr, active, max_steps)
                steps += 1
                illegal += int(ill)
            errors.append(steps - hanoi_solver(s0))
            rates.append(illegal / steps)
        data.append([S, sum(errors) / len(errors)])
    assert k == len(calls)
    return data, rates, np.array(actions), np.array(mms)


@pytest.mark.parametrize("name", ACTING)
def test_get_results_oracle(oracle, name):
    g = golden(f"acting_{name}.npz")
    np.random.seed(int(g["seed"]))
    data, _, actions, mms = _oracle_episodes(oracle, g, [int(b) for b in g["budgets"]], int(g["episodes"]),
                                            int(g["start"]) >= 0, int(g["init_state_idx"]), float(g["temperature"]))
    assert data == g["data"].tolist()
    assert np.array_equal(actions, g["actions"]) and np.array_equal(mms, g["mm"])
    assert np.array_equal(np.random.random_sample(4), g["post_rng"]), "RNG stream position differs"


@pytest.mark.parametrize("name", ILLEGAL)
def test_illegal_move_rate_oracle(oracle, name):
    g = golden(f"illegal_{name}.npz")
    np.random.seed(int(g["seed"]))
    _, rates, actions, _ = _oracle_episodes(oracle, g, [int(g["n_sims"])], int(g["episodes"]), bool(g["fixed_start"]),
                                            int(g["init_state_idx"]), float(g["temperature"]))
    assert float(np.mean(rates)) == float(g["mean"])
    assert float(np.std(rates, ddof=1) / np.sqrt(len(rates))) == float(g["sem"])
    assert np.array_equal(actions, g["actions"])
    assert np.array_equal(np.random.random_sample(4), g["post_rng"])


def test_start_states_and_labels():
    """acting_ablations.py:49-68: ES / MS / LS are 7 / 3 / 1 optimal moves from the goal"""
    from muzero_hanoi_amd.hanoi_utils import hanoi_solver
    from muzero_hanoi_amd.selfplay import START_STATES

    assert [hanoi_solver(START_STATES[k]) for k in ("ES", "MS", "LS")] == [7, 3, 1]


# ------------------------------------------------------------------------------------------- GPU
def _dropin_env(g):
    from muzero_hanoi_amd.env import TowersOfHanoi

    return TowersOfHanoi(N=int(g["n"]), max_steps=int(g["max_steps"]))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ACTING)
def test_get_results_dropin_gpu(name):
    from muzero_hanoi_amd import acting
    from muzero_hanoi_amd.mcts import MCTS, RecordedNetwork

    g = golden(f"acting_{name}.npz")
    env = _dropin_env(g)
    start = None if int(g["start"]) < 0 else int(g["start"])
    assert acting.get_starting_state(env, start) == str(g["start_label"])
    budgets = [int(b) for b in g["budgets"]]
    mcts = MCTS(discount=0.8, root_dirichlet_alpha=0.25, n_simulations=budgets[0], batch_s=256, device="cpu")
    net = RecordedNetwork(recorded_calls(g), int(g["n"]))
    np.random.seed(int(g["seed"]))
    data = acting.get_results(env, start, net, mcts, int(g["episodes"]), budgets, float(g["temperature"]))
    assert data == g["data"].tolist()
    assert net.cursor == len(g["run_S"])
    assert (mcts.min_max_stats.maximum, mcts.min_max_stats.minimum) == tuple(g["mm"][-1])
    assert np.array_equal(np.random.random_sample(4), g["post_rng"]), "RNG stream position differs"


@pytest.mark.gpu
@pytest.mark.parametrize("name", ILLEGAL)
def test_illegal_move_rate_dropin_gpu(name):
    from muzero_hanoi_amd import acting
    from muzero_hanoi_amd.mcts import MCTS, RecordedNetwork

    g = golden(f"illegal_{name}.npz")
    env = _dropin_env(g)
    env.init_state_idx = int(g["init_state_idx"])
    mcts = MCTS(discount=0.8, root_dirichlet_alpha=0.25, n_simulations=int(g["n_sims"]), batch_s=1, device="cpu")
    net = RecordedNetwork(recorded_calls(g), int(g["n"]))
    np.random.seed(int(g["seed"]))
    mean, sem = acting.illegal_move_rate(env, net, mcts, episodes=int(g["episodes"]),
                                         temperature=float(g["temperature"]), fixed_start=bool(g["fixed_start"]))
    assert (mean, sem) == (float(g["mean"]), float(g["sem"]))
    assert np.array_equal(np.random.random_sample(4), g["post_rng"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ACTING)
def test_evaluate_sequential_gpu(name):
    """the batched evaluator in the reference's schedule reproduces get_results"""
    from muzero_hanoi_amd.mcts import RecordedNetwork
    from muzero_hanoi_amd.selfplay import evaluate

    g = golden(f"acting_{name}.npz")
    start = None if int(g["start"]) < 0 else str(g["start_label"])
    net = RecordedNetwork(recorded_calls(g), int(g["n"]))
    np.random.seed(int(g["seed"]))
    out = evaluate(net, int(g["n"]), [int(b) for b in g["budgets"]], episodes=int(g["episodes"]), start=start,
                   max_steps=int(g["max_steps"]), temperature=float(g["temperature"]), sequential=True)
    assert out["data"] == g["data"].tolist()
    assert tuple(out["minmax"][0]) == tuple(g["mm"][-1])
    assert np.array_equal(np.random.random_sample(4), g["post_rng"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ILLEGAL)
def test_evaluate_illegal_rate_gpu(name):
    """per-episode-mean illegal rate and its standard error (not the pooled rate)"""
    from muzero_hanoi_amd.mcts import RecordedNetwork
    from muzero_hanoi_amd.selfplay import evaluate

    g = golden(f"illegal_{name}.npz")
    start = int(g["init_state_idx"]) if bool(g["fixed_start"]) else None
    net = RecordedNetwork(recorded_calls(g), int(g["n"]))
    np.random.seed(int(g["seed"]))
    out = evaluate(net, int(g["n"]), [int(g["n_sims"])], episodes=int(g["episodes"]), start=start,
                   max_steps=int(g["max_steps"]), temperature=float(g["temperature"]), sequential=True)
    assert out["illegal"][0][1:] == [float(g["mean"]), float(g["sem"])]
