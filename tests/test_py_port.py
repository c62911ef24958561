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
