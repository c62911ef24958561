"""Pin the CPU-baseline port (oracle/py_port.py) against the reference's own traces."""
import numpy as np
import pytest

from conftest import GOLDEN, REPLAY_CASES, golden
from oracle import py_port


def _roots(g):
    return range(g["obs"].shape[0])


@pytest.mark.parametrize("case", [c for c in REPLAY_CASES if c in ("n3s25_sto", "n4s50_sto", "n4s50_shared", "n4s50_det_t0", "n3s25_mc")])
def test_port_replay_bit_exact(case):
    g = golden(f"replay_{case}.npz")
    np.random.seed(int(g["seed"]))
    S = int(g["s"])
    m = None
    for b in _roots(g):
        if m is None or not int(g["shared"]):
            m = py_port.PortMCTS(float(g["discount"]), float(g["alpha"]), S)
        net = py_port.ReplayNet(g["out_pi"][b, 0], g["out_pi"][b, 1:], g["out_rwd"][b, 1:], g["out_v"][b, 1:])
        a, pi, q, visits = m.run_mcts(g["obs"][b], net, float(g["temperature"]), bool(g["deterministic"]))
        assert np.array_equal(visits, g["visits"][b])
        assert q == g["rootQ"][b] and a == g["action"][b] and np.array_equal(pi, g["pi"][b])


@pytest.mark.parametrize("case", ["n3s25_sto", "n4s50_sto"])
def test_port_end_to_end_equals_reference(case):
    """Same torch batch-1 ops as the reference -> identical visit counts end to end."""
    g = golden(f"replay_{case}.npz")
    z = np.load(f"{GOLDEN}/weights_N{int(g['n'])}_s0.npz")
    net = py_port.PortNet({k: z[k] for k in py_port.WEIGHT_KEYS})
    np.random.seed(int(g["seed"]))
    for b in _roots(g):
        m = py_port.PortMCTS(float(g["discount"]), float(g["alpha"]), int(g["s"]))
        a, pi, q, visits = m.run_mcts(g["obs"][b], net, float(g["temperature"]), bool(g["deterministic"]))
        assert np.array_equal(visits, g["visits"][b])
        assert q == g["rootQ"][b] and a == g["action"][b]


@pytest.mark.parametrize("n", [3, 4])
def test_port_hanoi_exhaustive(n):
    """PortHanoi (the host env step the env bench times as the reference's) equals the reference's exhaustive
    transition tables: next state, the moved state its observation encodes, reward, done and illegal"""
    g = golden(f"env_N{n}.npz")
    env = py_port.PortHanoi(n, 10**9)
    idx = {s: i for i, s in enumerate(env.states)}
    for i, st in enumerate(env.states):
        for a in range(6):
            env.reset_check, env.step_counter, env.c_state = True, 0, st
            obs, rwd, done, ill = env.step(a)
            moved = tuple(int(x) for x in np.argmax(obs.reshape(n, 3), 1))
            assert idx[env.c_state] == g["next_state"][i, a] and idx[moved] == g["moved_state"][i, a]
            assert rwd == g["reward"][i, a] and done == g["done"][i, a] and ill == g["illegal"][i, a]
