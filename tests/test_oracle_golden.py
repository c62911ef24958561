"""Pin the CPU oracle against the golden fixtures generated from the reference itself.

Bar: bit-exact for env / solver / tree arithmetic (replayed network outputs); logits within 1e-5
(north_star); transformed value/reward within 2e-3 (torch-CPU sqrt is not correctly rounded and
the signed-parabolic transform amplifies 1 ulp by ~500x).
"""
import math

import numpy as np
import pytest

from conftest import REPLAY_CASES, golden
from muzero_hanoi_amd import rng as mrng


def _states(n):
    idx = np.arange(3 ** n)
    return np.stack([(idx // 3 ** (n - 1 - d)) % 3 for d in range(n)], 1).astype(np.uint8)


def _index(st):
    v = 0
    for s in st:
        v = v * 3 + int(s)
    return v


@pytest.mark.parametrize("n", [3, 4, 7])
def test_env_exhaustive(oracle, n):
    g = golden(f"env_N{n}.npz")
    states = _states(n)
    code_to_rwd = {0: 0.0, 1: 100.0, -1: -100 / 1000}
    for i, st in enumerate(states):
        assert oracle.legal_mask(st) == sum(int(g["legal"][i, a]) << a for a in range(6))
        for a in range(6):
            code, new, moved, ctr, active, done, ill = oracle.env_step(st, a, 0, 1, 10**9)
            assert _index(moved) == g["moved_state"][i, a]
            assert _index(new) == g["next_state"][i, a]
            assert code_to_rwd[code] == g["reward"][i, a]
            assert done == g["done"][i, a] and ill == g["illegal"][i, a]


def test_env_maxsteps_sequences(oracle):
    g = golden("env_maxsteps.npz")
    for row in g["rows"]:
        n, max_steps, _, before, ctr_before, a, moved, after, rwd, done, ill, ctr_after, rc = row
        st = _states(int(n))[int(before)]
        code, new, mv, ctr, active, d, il = oracle.env_step(st, int(a), int(ctr_before), 1, int(max_steps))
        assert _index(mv) == moved and _index(new) == after
        assert {0: 0.0, 1: 100.0, -1: -0.1}[code] == rwd
        assert (d, il, ctr, active) == (done, ill, ctr_after, rc)
    # step before reset -> error code (AssertionError in the reference, env/hanoi.py:49)
    assert oracle.env_step(_states(3)[0], 0, 0, 0, 10)[0] == -2


@pytest.mark.parametrize("n", [3, 4, 7])
def test_solver(oracle, n):
    g = golden(f"solver_N{n}.npz")
    states = _states(n)
    for i, st in enumerate(states):
        assert oracle.hanoi_solver(st) == g["moves"][i]
        assert oracle.hanoi_solver(st, 0) == g["moves_goal0"][i]


def test_expf_accuracy(oracle):
    xs = np.concatenate([np.linspace(-87, 0, 20001, dtype=np.float32),
                         -np.random.RandomState(0).exponential(3, 5000).astype(np.float32)])
    xs = xs[xs >= -87]
    ours = np.array([oracle.expf(x) for x in xs], np.float32)
    ref = np.exp(xs.astype(np.float64))
    rel = np.abs(ours - ref) / ref
    assert rel.max() < 3 * 2.0 ** -23, rel.max()


def test_signed_parabolic_matches_restated_order(oracle):
    """The oracle's op order == the reference's fp32 op order with a correctly rounded sqrt."""
    rs = np.random.RandomState(1)
    xs = np.concatenate([rs.uniform(-16, 16, 4000), [0.0, 16.0, -16.0, 1e-6]]).astype(np.float32)
    f32 = np.float32
    for x in xs:
        t = f32(f32(1.001) + np.abs(x))
        t = f32(f32(0.004) * t)
        t = f32(f32(1) + t)
        t = np.sqrt(t)
        t = f32(t / f32(2))
        t = f32(t / f32(0.001))
        z = f32(t - f32(500.0))
        want = f32(np.sign(x) * f32(z * z - f32(1)))
        got = np.float32(oracle.lib().orc_signed_parabolic(float(x)))
        assert got.tobytes() == want.tobytes(), (x, got, want)


def test_ucb_table_matches_python():
    from oracle import oracle as orc

    t = orc.ucb_table(300)
    for n in range(300):
        ref = (math.log((n + 19652 + 1) / 19652) + 1.25) * math.sqrt(n)
        assert t[n] == ref


@pytest.mark.parametrize("name", ["mlp_N3_s0", "mlp_N4_s0", "mlp_N4_s1", "mlp_N7_s0", "mlp_N3_s0_mc"])
def test_mlp_vs_reference(oracle, name):
    g = golden(name + ".npz")
    wname = name.replace("mlp_", "weights_")
    w, in_dim, support = oracle.load_weights_npz(f"{__import__('conftest').GOLDEN}/{wname}.npz")
    flat = oracle.flat_weights(w)
    ii = oracle.initial_inference(flat, in_dim, support, g["x"])
    np.testing.assert_allclose(ii["policy_logits"], g["ii_policy_logits"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(ii["value_logits"], g["ii_value_logits"].reshape(ii["value_logits"].shape), atol=1e-5, rtol=0)
    np.testing.assert_allclose(ii["h"], g["ii_h"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(ii["pi"], g["ii_pi"], atol=1e-6, rtol=0)
    np.testing.assert_allclose(ii["value"], g["ii_value"], atol=2e-3, rtol=0)
    assert np.all(ii["reward"] == 0.0)
    ri = oracle.recurrent_inference(flat, in_dim, support, g["h_in"], g["a_in"])
    np.testing.assert_allclose(ri["policy_logits"], g["ri_policy_logits"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(ri["value_logits"], g["ri_value_logits"].reshape(ri["value_logits"].shape), atol=1e-5, rtol=0)
    np.testing.assert_allclose(ri["reward_logits"], g["ri_rwd_logits"].reshape(ri["reward_logits"].shape), atol=1e-5, rtol=0)
    np.testing.assert_allclose(ri["h"], g["ri_h"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(ri["pi"], g["ri_pi"], atol=1e-6, rtol=0)
    np.testing.assert_allclose(ri["value"], g["ri_value"], atol=2e-3, rtol=0)
    np.testing.assert_allclose(ri["reward"], g["ri_rwd"], atol=2e-3, rtol=0)


def replay_inputs(g):
    """Recorded network outputs of the reference run -> the oracle/kernel replay arrays."""
    return dict(root_pi=g["out_pi"][:, 0], pi=g["out_pi"][:, 1:], rwd=g["out_rwd"][:, 1:].astype(np.float32),
                value=g["out_v"][:, 1:].astype(np.float32))


def replay_draws(g):
    np.random.seed(int(g["seed"]))
    B = g["obs"].shape[0]
    if int(g["shared"]):
        return [mrng.predraw(1, deterministic=bool(g["deterministic"]), alpha=float(g["alpha"])) for _ in range(B)]
    return mrng.predraw(B, deterministic=bool(g["deterministic"]), alpha=float(g["alpha"]))


@pytest.mark.parametrize("case", REPLAY_CASES)
def test_replay_tree_bit_exact(oracle, case):
    g = golden(f"replay_{case}.npz")
    S = int(g["s"])
    n = int(g["n"])
    det = bool(g["deterministic"])
    T = float(g["temperature"])
    rp = replay_inputs(g)
    # the recorded outputs are exact fp32 values (python floats from fp32 .item())
    assert np.all(rp["rwd"].astype(np.float64) == g["out_rwd"][:, 1:])
    B = g["obs"].shape[0]
    if int(g["shared"]):
        draws = replay_draws(g)
        mm = np.array([[-np.inf, np.inf]])
        outs = []
        for b in range(B):
            noise, tie, u = draws[b]
            o = oracle.search(n, S, g["obs"][b:b + 1], replay={k: v[b:b + 1] for k, v in rp.items()},
                              noise=noise, tie_idx=tie, action_u=u, temperature=T, deterministic=det,
                              minmax_in=mm, discount=float(g["discount"]))
            mm = np.stack([o["mm_max"], o["mm_min"]], 1)
            outs.append(o)
        out = {k: np.concatenate([o[k] for o in outs]) for k in outs[0]}
    else:
        noise, tie, u = replay_draws(g)
        if noise is not None:
            mixed = (np.float32(0.75) * g["out_pi"][:, 0]).astype(np.float64) + 0.25 * noise
            assert np.array_equal(mixed, g["noised"])
        out = oracle.search(n, S, g["obs"], replay=rp, noise=noise, tie_idx=tie, action_u=u,
                            temperature=T, deterministic=det, discount=float(g["discount"]))
    assert np.array_equal(out["visits"], g["visits"])
    assert np.array_equal(out["rootQ"], g["rootQ"])
    assert np.array_equal(out["mm_max"], g["mm_max"]) and np.array_equal(out["mm_min"], g["mm_min"])
    assert np.array_equal(out["pi"], g["pi"])
    assert np.array_equal(out["action"], g["action"])
    assert np.all(out["extra_ties"] == 0)
    for b in range(B):
        L = out["latent_len"][b]
        want = g["latent"][b]
        assert list(out["latent"][b][:L]) == [int(v) for v in want[want >= 0]]


@pytest.mark.parametrize("n", [3, 4, 7])
def test_hanoi_solver_dropin_host(n):
    """the scalar drop-in (host closed form) equals the reference's hanoi_solver on every state"""
    from muzero_hanoi_amd.hanoi_utils import hanoi_solver

    g = golden(f"solver_N{n}.npz")
    for i, st in enumerate(_states(n)):
        assert hanoi_solver(tuple(int(x) for x in st)) == g["moves"][i]
        assert hanoi_solver(tuple(int(x) for x in st), 0) == g["moves_goal0"][i]
