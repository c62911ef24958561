"""Play policy (MCTS/mcts.py:154-176) at non-integer exponents, and the invalid-temperature edge.

generate_play_policy raises visit counts to exp = max(1, min(5, 1/T)) with np.power on an int64
array.  For a non-integer exp NumPy's float64 power is vectorised (SVML on AVX-512 hosts, which
this container and the GPU box both are) and differs from libm's pow in the last bit for some
counts, so the product path takes those powers from the caller's NumPy (engine.pow_table, the
mzh_search_args.pow_table field) and the oracle does the same.  Fixtures: play_policy.npz,
replay_n4s50_sto_t03 / _t07 / replay_n3s25_sto_t09 (reference runs), bad_temperature.npz
(tests/golden/gen_golden.py).
"""
import math

import numpy as np
import pytest

from conftest import golden

KERNELS = ["coop", "wave", "wave16"]


def test_play_policy_fixture_oracle(oracle):
    """the oracle's play policy == the reference's generate_play_policy, bit for bit, on 600
    histograms x 13 temperatures (8 with a non-integer exponent)"""
    g = golden("play_policy.npz")
    for ti, t in enumerate(g["temps"]):
        for h, want in zip(g["visits"], g["pi"][ti]):
            _, pi = oracle.play_policy(h, float(t), True)
            assert np.array_equal(pi, want), (t, h)


def test_dropin_generate_play_policy():
    from muzero_hanoi_amd.mcts import MCTS

    g = golden("play_policy.npz")
    m = MCTS(0.8, 0.25, 1, 1, "cpu")
    for ti, t in enumerate(g["temps"]):
        got = np.array([m.generate_play_policy(h, float(t)) for h in g["visits"]])
        assert np.array_equal(got, g["pi"][ti]), t


def test_pow_table_is_numpys_power():
    """the table the engine hands to the kernel is the reference's np.power, element for element;
    how often libm's pow differs from it here is reported (0 on a host whose NumPy has no SIMD pow)"""
    from oracle import oracle as orc

    g = golden("play_policy.npz")
    diff = 0
    for ti, t in enumerate(g["temps"]):
        tab = orc.numpy_pow_table(200, float(t))
        e = max(1.0, min(5.0, 1.0 / float(t)))
        if tab is None:
            assert e == int(e)
            continue
        assert np.array_equal(tab, g["powers"][ti])
        diff += int(sum(math.pow(float(n), e) != tab[n] for n in range(201)))
    print(f"libm pow != NumPy power on {diff} of the fixture's table entries")


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("T", [0.3, 0.7, 0.9, 0.45, 0.999])
def test_play_policy_gpu_equals_numpy(kernel, T):
    """replayed searches over 3,000 roots at a non-integer exponent: the kernel's pi is exactly
    generate_play_policy(visits, T) as NumPy computes it, and the sampled action is
    choice(6, p=pi) with the pre-drawn uniform (legacy RandomState.choice arithmetic)"""
    import torch

    from muzero_hanoi_amd import rng
    from muzero_hanoi_amd.engine import Engine
    from muzero_hanoi_amd.mcts import MCTS

    B, S = 3000, 50
    g = np.random.default_rng(int(T * 1000))
    rp = dict(root_pi=g.dirichlet(np.full(6, 0.7), size=B).astype(np.float32),
              pi=g.dirichlet(np.full(6, 0.7), size=(B, S)).astype(np.float32),
              reward=g.normal(0, 0.05, (B, S)).astype(np.float32), value=g.normal(0, 0.5, (B, S)).astype(np.float32))
    noise, tie, u = rng.synthetic_draws(B, deterministic=False, alpha=0.25, seed=5)
    eng = Engine(4, S, B, 33)
    tt = lambda a: torch.tensor(np.asarray(a), device="cuda")
    o = eng.search(S, replay={k: tt(v) for k, v in rp.items()}, tie_idx=tt(tie), noise=tt(noise), action_u=tt(u),
                   temperature=T, deterministic=False, kernel=kernel)
    vis, pi, act = (o[k].cpu().numpy() for k in ("visits", "pi", "action"))
    m = MCTS(0.8, 0.25, S, 1, "cpu")
    want = np.array([m.generate_play_policy(v, T) for v in vis])
    assert np.array_equal(pi, want)
    for b in range(B):
        cdf = np.cumsum(want[b])
        cdf /= cdf[-1]
        assert act[b] == int(cdf.searchsorted(u[b], side="right"))


@pytest.mark.gpu
def test_invalid_temperature_state_after_raise():
    """MCTS.run_mcts with T outside [0, 1] between valid calls on one instance: like the reference
    it raises ValueError after the search, leaving MinMaxStats / latent_actions updated and the
    NumPy stream after the Dirichlet and tie draws but before the action draw"""
    from muzero_hanoi_amd.mcts import MCTS, RecordedNetwork

    g = golden("bad_temperature.npz")
    calls = [dict(root_pi=g["out_pi"][b][0], pi=g["out_pi"][b][1:], reward=g["out_rwd"][b][1:].astype(np.float32),
                  value=g["out_v"][b][1:].astype(np.float32)) for b in range(len(g["temps"]))]
    net = RecordedNetwork(calls, int(g["n"]))
    mcts = MCTS(discount=0.8, root_dirichlet_alpha=0.25, n_simulations=int(g["s"]), batch_s=1, device="cpu")
    np.random.seed(int(g["seed"]))
    for b, t in enumerate(g["temps"]):
        if g["raised"][b]:
            with pytest.raises(ValueError):
                mcts.run_mcts(g["obs"][b], net, float(t), False)
        else:
            action, pi, _ = mcts.run_mcts(g["obs"][b], net, float(t), False)
            assert action == g["action"][b] and np.array_equal(pi, g["pi"][b])
        assert mcts.min_max_stats.maximum == g["mm_max"][b] and mcts.min_max_stats.minimum == g["mm_min"][b]
        lat = [int(x.item()) for x in mcts.return_latent_actions()]
        want = g["latent"][b]
        assert lat == [int(v) for v in want[want >= 0]]
    assert np.array_equal(np.random.random_sample(4), g["post_rng"])
