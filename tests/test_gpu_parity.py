"""GPU parity: the HIP path (through the C ABI) against the oracle and the reference fixtures.

Bars (north_star): env transitions and visit counts bit-exact; logits within 1e-5 of the
reference (torch-CPU); against the oracle (same fp32 op order) the MLP is expected bit-exact.
"""
import numpy as np
import pytest
import torch

from conftest import GOLDEN, REPLAY_CASES, golden
from test_oracle_golden import _index, _states, replay_draws, replay_inputs

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def mzh():
    from muzero_hanoi_amd import _lib, engine

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    _lib.lib()
    return engine


def _engine(mzh, n, S, B, support=33, weights=None):
    eng = mzh.Engine(n, S, B, support)
    if weights is not None:
        eng.load_weights(weights)
    return eng


def _weights(oracle, name):
    w, in_dim, sup = oracle.load_weights_npz(f"{GOLDEN}/{name}.npz")
    return oracle.flat_weights(w), in_dim, sup


# ------------------------------------------------------------------------------------ env
@pytest.mark.parametrize("n", [3, 4, 7])
def test_env_step_exhaustive(mzh, n):
    g = golden(f"env_N{n}.npz")
    states = _states(n)
    S = len(states)
    st = torch.tensor(np.repeat(states, 6, axis=0), device=DEV)
    act = torch.tensor(np.tile(np.arange(6), S), dtype=torch.int32, device=DEV)
    ctr = torch.zeros(S * 6, dtype=torch.int32, device=DEV)
    active = torch.ones(S * 6, dtype=torch.uint8, device=DEV)
    moved = torch.empty_like(st)
    obs = torch.empty((S * 6, 3 * n), dtype=torch.float32, device=DEV)
    rew, done, ill = mzh.env_step(n, 10**9, st, act, ctr, active, moved=moved, obs=obs)
    torch.cuda.synchronize()
    st, moved, obs = st.cpu().numpy(), moved.cpu().numpy(), obs.cpu().numpy()
    rew, done, ill = rew.cpu().numpy(), done.cpu().numpy(), ill.cpu().numpy()
    code_to_rwd = {0: 0.0, 1: 100.0, -1: -100 / 1000}
    for i in range(S):
        for a in range(6):
            k = i * 6 + a
            assert _index(st[k]) == g["next_state"][i, a]
            assert _index(moved[k]) == g["moved_state"][i, a]
            assert code_to_rwd[int(rew[k])] == g["reward"][i, a]
            assert done[k] == g["done"][i, a] and ill[k] == g["illegal"][i, a]
            want = np.zeros(3 * n, np.float32)
            want[np.arange(n) * 3 + moved[k]] = 1
            assert np.array_equal(obs[k], want)
    mask = mzh.legal_mask(n, torch.tensor(states, device=DEV)).cpu().numpy()
    assert np.array_equal(mask, (g["legal"].astype(np.int64) << np.arange(6)).sum(1))
    sol = mzh.hanoi_solver_batch(n, torch.tensor(states, device=DEV)).cpu().numpy()
    assert np.array_equal(sol, golden(f"solver_N{n}.npz")["moves"])
    sol0 = mzh.hanoi_solver_batch(n, torch.tensor(states, device=DEV), goal_peg=0).cpu().numpy()
    assert np.array_equal(sol0, golden(f"solver_N{n}.npz")["moves_goal0"])


def test_env_maxsteps_and_assert(mzh):
    g = golden("env_maxsteps.npz")
    for row in g["rows"]:
        n, max_steps, _, before, ctr_before, a, moved, after, rwd, done, ill, ctr_after, rc = [int(v) if i != 8 else v for i, v in enumerate(row)]
        st = torch.tensor(_states(n)[before][None], device=DEV)
        mv = torch.empty_like(st)
        ctr = torch.tensor([ctr_before], dtype=torch.int32, device=DEV)
        active = torch.ones(1, dtype=torch.uint8, device=DEV)
        r, d, il = mzh.env_step(n, max_steps, st, torch.tensor([a], dtype=torch.int32, device=DEV), ctr, active, moved=mv)
        assert _index(st[0].cpu().numpy()) == after and _index(mv[0].cpu().numpy()) == moved
        assert {0: 0.0, 1: 100.0, -1: -0.1}[int(r.item())] == rwd
        assert (int(d.item()), int(il.item()), int(ctr.item()), int(active.item())) == (done, ill, ctr_after, rc)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    st = torch.zeros((2, 3), dtype=torch.uint8, device=DEV)
    r, d, il = mzh.env_step(3, 10, st, torch.tensor([0, 9], dtype=torch.int32, device=DEV),
                            torch.zeros(2, dtype=torch.int32, device=DEV),
                            torch.tensor([0, 1], dtype=torch.uint8, device=DEV), err=err)
    assert err.item() == 2 and r.tolist() == [-2, -2]


# ------------------------------------------------------------------------------------ MLP
@pytest.mark.parametrize("name", ["mlp_N3_s0", "mlp_N4_s0", "mlp_N4_s1", "mlp_N7_s0", "mlp_N3_s0_mc"])
def test_mlp_vs_reference_and_oracle(mzh, oracle, name):
    g = golden(name + ".npz")
    flat, in_dim, sup = _weights(oracle, name.replace("mlp_", "weights_"))
    n = in_dim // 3
    eng = _engine(mzh, n, 4, 64, sup, flat)
    ii = {k: v.cpu().numpy() for k, v in eng.initial_inference(torch.tensor(g["x"], device=DEV)).items()}
    ri = {k: v.cpu().numpy() for k, v in eng.recurrent_inference(torch.tensor(g["h_in"], device=DEV),
                                                                  torch.tensor(g["a_in"], device=DEV)).items()}
    # vs the reference (torch-CPU): logits within 1e-5 (north_star); transformed scalars 2e-3
    np.testing.assert_allclose(ii["policy_logits"], g["ii_policy_logits"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(ii["value_logits"], g["ii_value_logits"].reshape(ii["value_logits"].shape), atol=1e-5, rtol=0)
    np.testing.assert_allclose(ii["h"], g["ii_h"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(ii["pi"], g["ii_pi"], atol=1e-6, rtol=0)
    np.testing.assert_allclose(ii["value"], g["ii_value"], atol=2e-3, rtol=0)
    np.testing.assert_allclose(ri["policy_logits"], g["ri_policy_logits"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(ri["value_logits"], g["ri_value_logits"].reshape(ri["value_logits"].shape), atol=1e-5, rtol=0)
    np.testing.assert_allclose(ri["reward_logits"], g["ri_rwd_logits"].reshape(ri["reward_logits"].shape), atol=1e-5, rtol=0)
    np.testing.assert_allclose(ri["h"], g["ri_h"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(ri["value"], g["ri_value"], atol=2e-3, rtol=0)
    np.testing.assert_allclose(ri["reward"], g["ri_rwd"], atol=2e-3, rtol=0)
    # vs the oracle: identical fp32 operation order -> identical bits
    oi = oracle.initial_inference(flat, in_dim, sup, g["x"])
    orr = oracle.recurrent_inference(flat, in_dim, sup, g["h_in"], g["a_in"])
    for k in ("h", "pi", "value", "policy_logits", "value_logits"):
        assert np.array_equal(ii[k], oi[k]), f"initial {k}: max |d| = {np.abs(ii[k] - oi[k]).max()}"
    for k in ("h", "pi", "value", "reward", "policy_logits", "value_logits", "reward_logits"):
        assert np.array_equal(ri[k], orr[k]), f"recurrent {k}: max |d| = {np.abs(ri[k] - orr[k]).max()}"


@pytest.mark.parametrize("B", [1, 17, 300, 9000])
def test_mlp_batch_sizes_vs_oracle(mzh, oracle, B):
    flat, in_dim, sup = _weights(oracle, "weights_N4_s0")
    rs = np.random.RandomState(B)
    x = np.zeros((B, 12), np.float32)
    st = rs.randint(0, 3, (B, 4))
    x[np.arange(B)[:, None], np.arange(4) * 3 + st] = 1
    h = rs.uniform(0, 1, (B, 64)).astype(np.float32)
    a = rs.randint(0, 6, B).astype(np.int32)
    eng = _engine(mzh, 4, 4, B, 33, flat)
    ii = eng.initial_inference(torch.tensor(x, device=DEV))
    ri = eng.recurrent_inference(torch.tensor(h, device=DEV), torch.tensor(a, device=DEV))
    oi = oracle.initial_inference(flat, in_dim, sup, x)
    orr = oracle.recurrent_inference(flat, in_dim, sup, h, a)
    for k in ("h", "pi", "value"):
        assert np.array_equal(ii[k].cpu().numpy(), oi[k])
    for k in ("h", "pi", "value", "reward"):
        assert np.array_equal(ri[k].cpu().numpy(), orr[k])


def _confident_heads(oracle):
    """weights_N4_s0 with the policy / value / reward output layers scaled (random-init logit
    spreads ~0.2-0.5) so that most rows' logits spread beyond the softmax heads' exact-division
    range (arguments < -65 take the IEEE fallback)"""
    w, in_dim, sup = oracle.load_weights_npz(f"{GOLDEN}/weights_N4_s0.npz")
    w = {k: v.copy() for k, v in w.items()}
    for k, scale in (("policy_net.2", 250.0), ("value_net.2", 250.0), ("rwd_net.2", 500.0)):
        w[k + ".weight"] *= np.float32(scale)
        w[k + ".bias"] *= np.float32(scale)
    return oracle.flat_weights(w), in_dim, sup


def test_softmax_fallback_confident_heads_vs_oracle(mzh, oracle):
    """A trained network's confident heads: logits more than 65 below the row maximum send the
    softmax's division to the IEEE fallback (mzh_device.h heads).  pi, value and reward stay
    bit-identical to the oracle for initial and recurrent inference."""
    flat, in_dim, sup = _confident_heads(oracle)
    B = 600
    rs = np.random.RandomState(5)
    x = np.zeros((B, 12), np.float32)
    x[np.arange(B)[:, None], np.arange(4) * 3 + rs.randint(0, 3, (B, 4))] = 1
    h = rs.uniform(0, 1, (B, 64)).astype(np.float32)
    a = rs.randint(0, 6, B).astype(np.int32)
    oi = oracle.initial_inference(flat, in_dim, sup, x)
    orr = oracle.recurrent_inference(flat, in_dim, sup, h, a)
    spread = lambda l: (l.max(1, keepdims=True) - l).max(1)
    assert (spread(oi["value_logits"]) > 65).mean() > 0.5 and (spread(orr["reward_logits"]) > 65).mean() > 0.5
    assert (spread(orr["policy_logits"]) > 65).any()
    eng = _engine(mzh, 4, 4, B, 33, flat)
    ii = eng.initial_inference(torch.tensor(x, device=DEV))
    ri = eng.recurrent_inference(torch.tensor(h, device=DEV), torch.tensor(a, device=DEV))
    for k in ("h", "pi", "value", "policy_logits", "value_logits"):
        assert np.array_equal(ii[k].cpu().numpy(), oi[k]), k
    for k in ("h", "pi", "value", "reward", "policy_logits", "value_logits", "reward_logits"):
        assert np.array_equal(ri[k].cpu().numpy(), orr[k]), k


# ------------------------------------------------------------------------------------ search
KERNELS = ["coop", "wave", "wave16"]
# MLP searches: also the two-workgroups-per-CU cooperative form (replay searches have no such form)
# and the latency kernel (one root per workgroup, mzh_one.hip)
KERNELS_MLP = KERNELS + ["occ2", "one"]


def _forced_fits(kernel, support, S):
    """whether a forced kernel can serve an S-simulation search (the two-workgroups-per-CU kernel: its LDS twice
    per CU; the latency kernel: its LDS tree and tables beside the output layers)"""
    from muzero_hanoi_amd import _lib, engine

    try:
        _lib.search_plan(support, 64, S, engine.search_flags(kernel))
        return True
    except RuntimeError:
        return False


@pytest.mark.parametrize("kernel", KERNELS_MLP)
def test_search_confident_heads_vs_oracle(mzh, oracle, kernel):
    """the fused searches with confident heads (softmax IEEE fallback inside the search kernels'
    heads) == the oracle's, every output bit for bit"""
    flat, in_dim, sup = _confident_heads(oracle)
    B, S, n = 300, 25, 4
    obs, noise, tie, u = _random_search_inputs(B, n, 77)
    eng = _engine(mzh, n, S, B, sup, flat)
    tt = lambda a: torch.tensor(np.asarray(a), device=DEV)
    o = eng.search(S, obs=tt(obs), tie_idx=tt(tie), noise=tt(noise), action_u=tt(u), temperature=1.0, kernel=kernel)
    o = {k: v.cpu().numpy() for k, v in o.items() if not k.startswith("_")}
    ref = oracle.search(n, S, obs, flat=flat, support=sup, noise=noise, tie_idx=tie, action_u=u, temperature=1.0)
    for k, rk in (("visits", "visits"), ("root_q", "rootQ"), ("action", "action"), ("sel_steps", "sel_steps"),
                  ("extra_ties", "extra_ties")):
        assert np.array_equal(o[k], ref[rk]), k


def _tiny_latent_gap(oracle):
    """weights_N4_s0 with the dynamics output layer made constant: h' = its bias, one unit 2^-110
    above the row minimum.  That unit's Markstein quotient in the latent normalisation flags `slow`
    (a numerator below 2^-100), so every kernel takes its exact-division rerun -- in the
    cooperative kernels the pass that runs after rwd0's MFMA chain (mzh_mlp_recurrent_body)"""
    w, in_dim, sup = oracle.load_weights_npz(f"{GOLDEN}/weights_N4_s0.npz")
    w = {k: v.copy() for k, v in w.items()}
    w["dynamic_net.2.weight"][:] = 0.0
    b = np.random.RandomState(11).uniform(0.25, 1.0, 64).astype(np.float32)
    b[3], b[17] = 0.0, np.float32(2.0 ** -110)
    w["dynamic_net.2.bias"][:] = b
    return oracle.flat_weights(w), in_dim, sup


def test_normalisation_exact_rerun_vs_oracle(mzh, oracle):
    """recurrent_inference with a latent unit 2^-110 above the row minimum == the oracle bit for bit"""
    flat, in_dim, sup = _tiny_latent_gap(oracle)
    B = 300
    rs = np.random.RandomState(6)
    h = rs.uniform(0, 1, (B, 64)).astype(np.float32)
    a = rs.randint(0, 6, B).astype(np.int32)
    orr = oracle.recurrent_inference(flat, in_dim, sup, h, a)
    assert (orr["h"] > 0).any() and (orr["h"][orr["h"] > 0] < 2.0 ** -100).any()  # the tiny quotient
    eng = _engine(mzh, 4, 4, B, 33, flat)
    ri = eng.recurrent_inference(torch.tensor(h, device=DEV), torch.tensor(a, device=DEV))
    for k in ("h", "pi", "value", "reward"):
        assert np.array_equal(ri[k].cpu().numpy(), orr[k]), k


@pytest.mark.parametrize("kernel,tile", [("coop", 16), ("coop", 32), ("wave", None), ("wave16", None), ("occ2", None)])
def test_search_normalisation_exact_rerun_vs_oracle(mzh, oracle, kernel, tile):
    """the fused searches with every expansion's latent normalised by the exact-division rerun ==
    the oracle's, every output bit for bit (both cooperative tiles and the wave kernels)"""
    flat, in_dim, sup = _tiny_latent_gap(oracle)
    B, S, n = 100, 12, 4
    obs, noise, tie, u = _random_search_inputs(B, n, 78)
    eng = _engine(mzh, n, S, B, sup, flat)
    tt = lambda a: torch.tensor(np.asarray(a), device=DEV)
    o = eng.search(S, obs=tt(obs), tie_idx=tt(tie), noise=tt(noise), action_u=tt(u), temperature=1.0, kernel=kernel,
                   tile=tile)
    o = {k: v.cpu().numpy() for k, v in o.items() if not k.startswith("_")}
    ref = oracle.search(n, S, obs, flat=flat, support=sup, noise=noise, tie_idx=tie, action_u=u, temperature=1.0)
    for k, rk in (("visits", "visits"), ("root_q", "rootQ"), ("action", "action"), ("sel_steps", "sel_steps"),
                  ("extra_ties", "extra_ties")):
        assert np.array_equal(o[k], ref[rk]), k


def _run_replay_case(mzh, g, kernel=None):
    S, n = int(g["s"]), int(g["n"])
    det, T = bool(g["deterministic"]), float(g["temperature"])
    rp = replay_inputs(g)
    B = g["obs"].shape[0]
    eng = _engine(mzh, n, max(S, 1), B, 33 if int(g["td"]) else 1)
    tt = lambda a, dt=None: None if a is None else torch.tensor(np.asarray(a), dtype=dt, device=DEV)
    if int(g["shared"]):
        draws = replay_draws(g)
        mm = torch.tensor([[-np.inf, np.inf]], dtype=torch.float64, device=DEV)
        outs = []
        for b in range(B):
            noise, tie, u = draws[b]
            o = eng.search(S, replay={k: tt(v[b:b + 1]) for k, v in dict(root_pi=rp["root_pi"], pi=rp["pi"], reward=rp["rwd"], value=rp["value"]).items()},
                           tie_idx=tt(tie), noise=tt(noise), action_u=tt(u), minmax_in=mm,
                           temperature=T, deterministic=det, discount=float(g["discount"]), kernel=kernel)
            mm = o["minmax"].clone()
            outs.append({k: v.cpu().numpy() for k, v in o.items() if not k.startswith("_")})
        return {k: np.concatenate([o[k] for o in outs]) for k in outs[0]}
    noise, tie, u = replay_draws(g)
    o = eng.search(S, replay=dict(root_pi=tt(rp["root_pi"]), pi=tt(rp["pi"]), reward=tt(rp["rwd"]), value=tt(rp["value"])),
                   tie_idx=tt(tie), noise=tt(noise), action_u=tt(u), temperature=T, deterministic=det,
                   discount=float(g["discount"]), kernel=kernel)
    return {k: v.cpu().numpy() for k, v in o.items() if not k.startswith("_")}


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("case", REPLAY_CASES)
def test_search_replay_bit_exact_vs_reference(mzh, case, kernel):
    g = golden(f"replay_{case}.npz")
    out = _run_replay_case(mzh, g, kernel)
    assert np.array_equal(out["visits"], g["visits"])
    assert np.array_equal(out["root_q"], g["rootQ"])
    assert np.array_equal(out["minmax"][:, 0], g["mm_max"]) and np.array_equal(out["minmax"][:, 1], g["mm_min"])
    assert np.array_equal(out["pi"], g["pi"])
    assert np.array_equal(out["action"], g["action"])
    assert np.all(out["extra_ties"] == 0)
    for b in range(g["obs"].shape[0]):
        L = out["latent_len"][b]
        want = g["latent"][b]
        assert list(out["latent"][b][:L]) == [int(v) for v in want[want >= 0]]


@pytest.mark.parametrize("kernel", KERNELS_MLP)
@pytest.mark.parametrize("case", [c for c in REPLAY_CASES if "shared" not in c])
def test_search_mlp_end_to_end_vs_oracle(mzh, oracle, case, kernel):
    """Full fused search (MLP on MFMA) == oracle search with the same weights, bit for bit."""
    g = golden(f"replay_{case}.npz")
    S, n, td = int(g["s"]), int(g["n"]), int(g["td"])
    flat, in_dim, sup = _weights(oracle, f"weights_N{n}_s{int(g['wseed'])}{'' if td else '_mc'}")
    det, T = bool(g["deterministic"]), float(g["temperature"])
    noise, tie, u = replay_draws(g)
    B = g["obs"].shape[0]
    eng = _engine(mzh, n, S, B, sup, flat)
    tt = lambda a: None if a is None else torch.tensor(np.asarray(a), device=DEV)
    kw = dict(obs=tt(g["obs"].astype(np.float32)), tie_idx=tt(tie), noise=tt(noise), action_u=tt(u), temperature=T,
              deterministic=det, discount=float(g["discount"]), kernel=kernel)
    if kernel in ("occ2", "one") and not _forced_fits(kernel, sup, S):
        # a forced kernel that cannot serve the search is an error, never a silent fallback (mzh.h)
        with pytest.raises(RuntimeError, match="MZH_FLAG_COOP_OCC2" if kernel == "occ2" else "MZH_FLAG_KERNEL_ONE"):
            eng.search(S, **kw)
        return
    o = eng.search(S, **kw)
    o = {k: v.cpu().numpy() for k, v in o.items() if not k.startswith("_")}
    ref = oracle.search(n, S, g["obs"], flat=flat, support=sup, noise=noise, tie_idx=tie, action_u=u,
                        temperature=T, deterministic=det, discount=float(g["discount"]))
    assert np.array_equal(o["visits"], ref["visits"])
    assert np.array_equal(o["root_q"], ref["rootQ"])
    assert np.array_equal(o["pi"], ref["pi"]) and np.array_equal(o["action"], ref["action"])
    assert np.array_equal(o["sel_steps"], ref["sel_steps"])
    # and against the reference's own visit counts (torch-CPU network): the measured agreement is
    # every root of every fixture (tests/test_parity_corners.py pins it on the oracle, 58 / 58)
    agree = (o["visits"] == g["visits"]).all(1)
    assert agree.all(), f"{int(agree.sum())} / {len(agree)} histograms equal the reference's"


@pytest.mark.parametrize("kernel,tile", [("coop", None), ("coop", 16), ("coop", 32), ("wave", None), ("wave16", None),
                                         ("occ2", None), ("one", None)])
@pytest.mark.parametrize("B,S,n", [(40, 50, 4), (700, 25, 3), (9000, 8, 4), (300, 20, 7)])
def test_search_batched_vs_oracle_random_roots(mzh, oracle, B, S, n, kernel, tile):
    """Ragged batches (not multiples of the 16/32-root tile), both tile sizes forced and by
    default, vs the oracle."""
    flat, in_dim, sup = _weights(oracle, f"weights_N{n}_s0")
    rs = np.random.RandomState(B + S)
    st = rs.randint(0, 3, (B, n))
    obs = np.zeros((B, 3 * n), np.float32)
    obs[np.arange(B)[:, None], np.arange(n) * 3 + st] = 1
    from muzero_hanoi_amd import rng

    noise, tie, u = rng.synthetic_draws(B, deterministic=False, alpha=0.25, seed=B)
    eng = _engine(mzh, n, S, B, sup, flat)
    tt = lambda a: torch.tensor(np.asarray(a), device=DEV)
    o = eng.search(S, obs=tt(obs), tie_idx=tt(tie), noise=tt(noise), action_u=tt(u), temperature=1.0, kernel=kernel,
                   tile=tile)
    o = {k: v.cpu().numpy() for k, v in o.items() if not k.startswith("_")}
    nchk = min(B, 300)
    ref = oracle.search(n, S, obs[:nchk], flat=flat, support=sup, noise=noise[:nchk], tie_idx=tie[:nchk],
                        action_u=u[:nchk], temperature=1.0)
    assert np.array_equal(o["visits"][:nchk], ref["visits"])
    assert np.array_equal(o["root_q"][:nchk], ref["rootQ"])
    assert np.array_equal(o["action"][:nchk], ref["action"])
    assert np.all(o["visits"].sum(1) == S)


def _random_search_inputs(B, n, seed):
    from muzero_hanoi_amd import rng

    rs = np.random.RandomState(seed)
    st = rs.randint(0, 3, (B, n))
    obs = np.zeros((B, 3 * n), np.float32)
    obs[np.arange(B)[:, None], np.arange(n) * 3 + st] = 1
    noise, tie, u = rng.synthetic_draws(B, deterministic=False, alpha=0.25, seed=seed)
    return obs, noise, tie, u


@pytest.mark.parametrize("B,S,n,td", [(40000, 50, 4, 1), (33000, 12, 3, 0)])
def test_search_wave_equals_coop_large_batch(mzh, oracle, B, S, n, td):
    """At the bench's batch sizes the two kernels agree on every output, bit for bit (ragged last
    workgroup included), and a sample of roots matches the oracle."""
    flat, in_dim, sup = _weights(oracle, f"weights_N{n}_s0{'' if td else '_mc'}")
    obs, noise, tie, u = _random_search_inputs(B, n, B + S)
    eng = _engine(mzh, n, S, B, sup, flat)
    tt = lambda a: torch.tensor(np.asarray(a), device=DEV)
    res = {}
    for kernel in KERNELS_MLP:
        o = eng.search(S, obs=tt(obs), tie_idx=tt(tie), noise=tt(noise), action_u=tt(u), temperature=1.0,
                       kernel=kernel)
        res[kernel] = {k: v.cpu().numpy() for k, v in o.items() if not k.startswith("_")}
    for kernel in KERNELS_MLP[1:]:
        for k in res["coop"]:
            assert np.array_equal(res["coop"][k], res[kernel][k], equal_nan=True), (kernel, k)
    idx = np.r_[0:32, B - 40:B]
    ref = oracle.search(n, S, obs[idx], flat=flat, support=sup, noise=noise[idx], tie_idx=tie[idx],
                        action_u=u[idx], temperature=1.0)
    assert np.array_equal(res["wave"]["visits"][idx], ref["visits"])
    assert np.array_equal(res["wave"]["root_q"][idx], ref["rootQ"])
    assert np.array_equal(res["wave"]["sel_steps"][idx], ref["sel_steps"])


@pytest.mark.parametrize("kernel,tile", [("coop", 16), ("coop", 32), ("wave", None), ("wave16", None)])
def test_search_deep_paths_replay(mzh, oracle, kernel, tile):
    """Replayed network outputs that drive the search down one long chain, deeper than every
    kernel's LDS-cached path levels (wave kernels 16; cooperative 32-root tile -- the 8,192-root
    shard of the 8-GPU headline -- 16; 16-root tile 32), so the backup's HBM branch for the deeper
    levels (mzh_tree.h, node.py:53-70) runs on every root: visits, root Q, min-max and the latent
    path vs the oracle."""
    B, S, n = 70, 120, 4
    g = np.random.default_rng(7)
    pi = np.full((B, S, 6), 0.002, np.float32)
    pi[:, :, 0] = 0.99
    root_pi = pi[:, 0].copy()
    value = (5.0 + g.normal(0, 0.1, (B, S))).astype(np.float32)
    rwd = g.normal(0, 0.01, (B, S)).astype(np.float32)
    rp = dict(root_pi=root_pi, pi=pi, rwd=rwd, value=value)
    obs = np.zeros((B, 3 * n), np.float32)
    obs[:, 0::3] = 1
    from muzero_hanoi_amd import rng

    noise, tie, u = rng.synthetic_draws(B, deterministic=True, alpha=0.0, seed=3)
    eng = _engine(mzh, n, S, B)
    tt = lambda a: None if a is None else torch.tensor(np.asarray(a), device=DEV)
    o = eng.search(S, replay=dict(root_pi=tt(root_pi), pi=tt(pi), reward=tt(rwd), value=tt(value)), tie_idx=tt(tie),
                   noise=None, action_u=None, temperature=1.0, deterministic=True, kernel=kernel, tile=tile)
    o = {k: v.cpu().numpy() for k, v in o.items() if not k.startswith("_")}
    ref = oracle.search(n, S, obs, replay=rp, tie_idx=tie, temperature=1.0, deterministic=True)
    # every root's paths average deeper than any LDS path cache (max depth 120 = S)
    assert (ref["sel_steps"] / S).min() > 32 and ref["latent_len"].max() == S
    assert np.array_equal(o["visits"], ref["visits"])
    assert np.array_equal(o["root_q"], ref["rootQ"])
    assert np.array_equal(o["minmax"][:, 0], ref["mm_max"]) and np.array_equal(o["minmax"][:, 1], ref["mm_min"])
    assert np.array_equal(o["latent_len"], ref["latent_len"])
    assert np.array_equal(o["latent"], ref["latent"])
    assert np.array_equal(o["sel_steps"], ref["sel_steps"])


# ------------------------------------------------------- BASELINE.json configs at full size
def _sample_idx(B, seed):
    """first 16, last 16 and 16 random roots of a batch"""
    mid = np.random.default_rng(seed).choice(np.arange(16, B - 16), 16, replace=False)
    return np.unique(np.r_[0:16, np.sort(mid), B - 16:B])


@pytest.mark.parametrize("B,S,n", [(4096, 50, 4),     # configs[1]
                                   (16384, 200, 4),   # configs[3]
                                   (32768, 100, 7),   # configs[4], one of its 8 shards
                                   (65536, 50, 4)])   # the metric's batch (bench.py, per GPU)
def test_search_baseline_configs_full_size(mzh, oracle, B, S, n):
    """Each BASELINE.json search config at its full per-GPU size through the kernel the engine picks
    for it: every root's visits sum to S, root Q is finite, and a sample of 48 roots (both ends of
    the batch + 16 random) equals the oracle bit for bit (visits, root Q, action, selection steps)."""
    flat, in_dim, sup = _weights(oracle, f"weights_N{n}_s0")
    obs, noise, tie, u = _random_search_inputs(B, n, 1000 + B + S)
    eng = _engine(mzh, n, S, B, sup, flat)
    tt = lambda a: torch.tensor(np.asarray(a), device=DEV)
    o = eng.search(S, obs=tt(obs), tie_idx=tt(tie), noise=tt(noise), action_u=tt(u), temperature=1.0)
    from muzero_hanoi_amd import _lib

    assert o["_plan"] == _lib.search_plan(sup, B, S)  # the host query names the launched instantiation
    o = {k: v.cpu().numpy() for k, v in o.items() if not k.startswith("_")}
    assert np.all(o["visits"].sum(1) == S)
    assert np.all(np.isfinite(o["root_q"]))
    assert np.all(o["sel_steps"] >= S)  # every simulation descends at least one edge
    idx = _sample_idx(B, B + S)
    ref = oracle.search(n, S, obs[idx], flat=flat, support=sup, noise=noise[idx], tie_idx=tie[idx],
                        action_u=u[idx], temperature=1.0)
    assert np.array_equal(o["visits"][idx], ref["visits"])
    assert np.array_equal(o["root_q"][idx], ref["rootQ"])
    assert np.array_equal(o["action"][idx], ref["action"])
    assert np.array_equal(o["sel_steps"][idx], ref["sel_steps"])


@pytest.mark.parametrize("B,S,n,W", [(65536, 50, 4, 8),    # configs[2]: 65,536 roots over 8 GPUs
                                     (262144, 100, 7, 8)])  # configs[4]: 262,144 roots over 8 GPUs
def test_search_sharded_equals_whole_batch(mzh, oracle, B, S, n, W):
    """The multi-GPU decomposition (bench.py / distributed.py: rank r searches roots
    [r*B/W, (r+1)*B/W) with the draws made in global root order) gives the same outputs as one
    launch over the whole batch, bit for bit, although shard and whole batch run different
    kernels (8,192-root shards: cooperative; 65,536 / 262,144 roots: wave)."""
    flat, in_dim, sup = _weights(oracle, f"weights_N{n}_s0")
    obs, noise, tie, u = _random_search_inputs(B, n, 2000 + B + S)
    tt = lambda a: torch.tensor(np.asarray(a), device=DEV)
    eng = _engine(mzh, n, S, B, sup, flat)
    whole = eng.search(S, obs=tt(obs), tie_idx=tt(tie), noise=tt(noise), action_u=tt(u), temperature=1.0)
    whole = {k: v.cpu().numpy() for k, v in whole.items() if not k.startswith("_")}
    eng.close()
    shard = B // W
    es = _engine(mzh, n, S, shard, sup, flat)
    for r in range(W):
        sl = slice(r * shard, (r + 1) * shard)
        o = es.search(S, obs=tt(obs[sl]), tie_idx=tt(tie[sl]), noise=tt(noise[sl]), action_u=tt(u[sl]),
                      temperature=1.0)
        o = {k: v.cpu().numpy() for k, v in o.items() if not k.startswith("_")}
        for k in ("visits", "root_q", "pi", "action", "sel_steps", "minmax", "extra_ties"):
            assert np.array_equal(o[k], whole[k][sl], equal_nan=True), (r, k)


@pytest.mark.parametrize("B,tile", [(4096, None), (8192, None), (600, 32)])
def test_search_caller_bounds_instantiation(mzh, oracle, B, tile):
    """The instantiation run_mcts and batched self-play launch (caller MinMaxStats bounds; the
    one-hot columns stay in LDS): fresh bounds give the same outputs as none, and a sample of roots
    with carried-over bounds equals the oracle bit for bit."""
    from muzero_hanoi_amd import _lib

    S, n = 50, 4
    flat, in_dim, sup = _weights(oracle, f"weights_N{n}_s0")
    obs, noise, tie, u = _random_search_inputs(B, n, 3000 + B)
    eng = _engine(mzh, n, S, B, sup, flat)
    tt = lambda a: torch.tensor(np.asarray(a), device=DEV)
    kw = dict(obs=tt(obs), tie_idx=tt(tie), noise=tt(noise), action_u=tt(u), temperature=1.0, tile=tile)
    base = eng.search(S, **kw)
    base = {k: v.cpu().numpy() for k, v in base.items() if not k.startswith("_")}
    fresh = np.tile(np.array([[-np.inf, np.inf]]), (B, 1))
    o = eng.search(S, minmax_in=tt(fresh), **kw)
    flags = mzh.search_flags(tile=tile)
    assert o["_plan"]["kernel"] == _lib.search_plan(sup, B, S, flags, minmax_in=True)["kernel"]
    assert o["_plan"]["kernel"].endswith("true, true, true>")  # one-hot in LDS + caller bounds
    o = {k: v.cpu().numpy() for k, v in o.items() if not k.startswith("_")}
    for k in ("visits", "root_q", "pi", "action", "sel_steps", "minmax", "extra_ties"):
        assert np.array_equal(o[k], base[k], equal_nan=True), k
    # carried-over bounds (a second search of the same MCTS instances)
    o2 = eng.search(S, minmax_in=tt(base["minmax"]), **kw)
    o2 = {k: v.cpu().numpy() for k, v in o2.items() if not k.startswith("_")}
    idx = _sample_idx(B, B)
    ref = oracle.search(n, S, obs[idx], flat=flat, support=sup, noise=noise[idx], tie_idx=tie[idx],
                        action_u=u[idx], temperature=1.0, minmax_in=base["minmax"][idx])
    assert np.array_equal(o2["visits"][idx], ref["visits"])
    assert np.array_equal(o2["root_q"][idx], ref["rootQ"])
    assert np.array_equal(o2["minmax"][idx, 0], ref["mm_max"]) and np.array_equal(o2["minmax"][idx, 1], ref["mm_min"])


# ------------------------------------------------- whole-batch oracle parity at BASELINE sizes
FULL_BATCH = [("c1_4096", None), ("c3_16384", None), ("c2_65536", None), ("c4_shard0of8", None),
              ("c2_shard7of8", None), ("c2_shard7of8", "occ2"), ("c2_shard7of8", "coop"), ("c1_4096", "occ2"),
              ("c1_4096_s1", None), ("c1_4096_s2", None), ("c1_4096_s3", None), ("c1_4096_s4", None),
              ("c1_4096_det", None), ("c1_4096_det", "wave16"), ("c1_4096", "one"), ("c1_4096_det", "one")]


def _first_diff(a, b):
    bad = np.flatnonzero(~(np.asarray(a) == np.asarray(b)).reshape(len(a), -1).all(1))
    return None if bad.size == 0 else (int(bad[0]), int(bad.size))


@pytest.mark.parametrize("tag,kernel", FULL_BATCH)
def test_search_full_batch_equals_oracle(mzh, tag, kernel):
    """EVERY root of each BASELINE.json search config at its full per-GPU size (configs[1] 4,096
    roots; configs[3] 16,384 x 200 sims; configs[2] 65,536 roots on one GPU; configs[4]'s rank-0
    shard at N=8, 32,768 7-disk roots x 100 sims), on bench.py's own inputs and reference-order
    draws, through the kernel the library picks, equals the C oracle's whole-batch outputs
    (tests/golden/gen_fullbatch.py; MCTS/mcts.py:34-126): visits, action, selection steps and extra
    ties root by root, root Q and MinMaxStats bit for bit through per-256-root SHA-256 digests.
    configs[1] also for seeds 1-4 and in the deterministic mode (alpha 0, argmax action)."""
    import sys

    sys.path.insert(0, GOLDEN)
    import gen_fullbatch as gf

    z = golden(f"full_{tag}.npz")
    n, S = int(z["n_disks"]), int(z["n_sims"])
    obs, noise, tie, u = gf.inputs(tag)
    assert np.array_equal(gf.inputs_sha(obs, noise, tie, u), z["inputs_sha"]), "regenerated inputs differ"
    flat, sup = gf.weights(n)
    B = len(obs)
    eng = _engine(mzh, n, S, B, sup, flat)
    tt = lambda a: None if a is None else torch.tensor(np.asarray(a), device=DEV)
    o = eng.search(S, obs=tt(obs), tie_idx=tt(tie), noise=tt(noise), action_u=tt(u), temperature=1.0,
                   deterministic=gf.deterministic(tag), discount=0.8, eps=0.25, kernel=kernel)
    kern = o["_plan"]["kernel"]
    if kernel in ("occ2", "one"):
        assert kern.startswith(f"mzh_search_{kernel}_kernel<"), kern
    o = {k: v.cpu().numpy() for k, v in o.items() if not k.startswith("_")}
    eng.close()
    for k, want in (("visits", z["visits"]), ("action", z["action"]), ("sel_steps", z["sel_steps"]),
                    ("extra_ties", z["extra_ties"])):
        d = _first_diff(o[k].astype(np.int64), want.astype(np.int64))
        assert d is None, f"{tag} ({kern}): {k} differs at root {d[0]} ({d[1]} of {B} roots)"
    sha = gf.block_sha(o["root_q"], o["minmax"])
    d = _first_diff(sha, z["rootq_minmax_sha"])
    assert d is None, f"{tag} ({kern}): root Q / MinMaxStats differ in 256-root block {d[0]} ({d[1]} blocks)"
    if "root_q" in z:
        assert np.array_equal(o["root_q"], z["root_q"]) and np.array_equal(o["minmax"], z["minmax"])


def test_search_configs4_whole_batch_equals_oracle(mzh):
    """configs[4] (7 disks, 262,144 roots, 100 sims) as ONE launch on one GPU (the wave kernel), every root
    against the C oracle: the eight N=8 shard fixtures (full_c4_shard{0..7}of8.npz) hold the oracle's
    outputs for all 262,144 roots in root order (MCTS/mcts.py:34-126)."""
    import sys

    sys.path.insert(0, GOLDEN)
    import gen_fullbatch as gf

    tags = [f"c4_shard{r}of8" for r in range(8)]
    parts = [gf.inputs(t) for t in tags]
    obs, noise, tie, u = (np.concatenate([p[i] for p in parts]) for i in range(4))
    zs = [golden(f"full_{t}.npz") for t in tags]
    n, S = int(zs[0]["n_disks"]), int(zs[0]["n_sims"])
    flat, sup = gf.weights(n)
    B = len(obs)
    assert B == 262144
    eng = _engine(mzh, n, S, B, sup, flat)
    tt = lambda a: torch.tensor(np.asarray(a), device=DEV)
    o = eng.search(S, obs=tt(obs), tie_idx=tt(tie), noise=tt(noise), action_u=tt(u), temperature=1.0,
                   deterministic=False, discount=0.8, eps=0.25)
    kern = o["_plan"]["kernel"]
    o = {k: v.cpu().numpy() for k, v in o.items() if not k.startswith("_")}
    eng.close()
    b = B // 8
    for r, (t, z) in enumerate(zip(tags, zs)):
        sl = slice(r * b, (r + 1) * b)
        for k, want in (("visits", z["visits"]), ("action", z["action"]), ("sel_steps", z["sel_steps"]),
                        ("extra_ties", z["extra_ties"])):
            d = _first_diff(o[k][sl].astype(np.int64), want.astype(np.int64))
            assert d is None, f"{t} ({kern}): {k} differs at root {r * b + d[0]} ({d[1]} roots)"
        d = _first_diff(gf.block_sha(o["root_q"][sl], o["minmax"][sl]), z["rootq_minmax_sha"])
        assert d is None, f"{t} ({kern}): root Q / MinMaxStats differ in 256-root block {d[0]} of the shard"


_LOCKSTEP_REF = {}


def _lockstep_ref(oracle, B, S, n, replay):
    """the oracle's per-simulation selection depths for the lockstep test's inputs (computed once)"""
    key = (B, S, n, replay)
    if key not in _LOCKSTEP_REF:
        flat, in_dim, sup = _weights(oracle, f"weights_N{n}_s0")
        obs, noise, tie, u = _random_search_inputs(B, n, 4321)
        g = np.random.default_rng(5)
        rp = dict(root_pi=g.dirichlet(np.full(6, 20.0), size=B).astype(np.float32),
                  pi=g.dirichlet(np.full(6, 20.0), size=(B, S)).astype(np.float32),
                  rwd=g.normal(0, 0.05, (B, S)).astype(np.float32), value=g.normal(0, 0.5, (B, S)).astype(np.float32))
        if replay:
            ref = oracle.search(n, S, obs, replay=rp, noise=noise, tie_idx=tie, action_u=u, temperature=1.0, depths=True)
        else:
            ref = oracle.search(n, S, obs, flat=flat, support=sup, noise=noise, tie_idx=tie, action_u=u,
                                temperature=1.0, depths=True)
        _LOCKSTEP_REF[key] = (flat, sup, obs, noise, tie, u, rp, ref)
    return _LOCKSTEP_REF[key]


@pytest.mark.parametrize("replay", [False, True])
@pytest.mark.parametrize("kernel,tile", [("coop", 16), ("coop", 32), ("occ2", None), ("wave", None), ("wave16", None),
                                         ("one", None)])
def test_search_lockstep_levels(mzh, oracle, kernel, tile, replay):
    """mzh_search_args.lockstep_levels (the select/backup latency model's input, bench.tree_latency_model):
    per lockstep group (a workgroup of the cooperative kernels, a wave of the wave kernels) the sum over
    simulations of its deepest selection below the root -- equal, group by group, to that sum over the
    oracle's per-simulation selection depths, in the fused search and in the replay instantiation (the one
    bench.py counts on); asking for it changes no other output"""
    from muzero_hanoi_amd import _lib

    if replay and kernel in ("occ2", "one"):
        pytest.skip(f"the {kernel} kernel has no replay instantiation")
    B, S, n = 600, 30, 4
    flat, sup, obs, noise, tie, u, rp, ref = _lockstep_ref(oracle, B, S, n, replay)
    eng = _engine(mzh, n, S, B, sup, flat)
    tt = lambda a: torch.tensor(np.asarray(a), device=DEV)
    kw = dict(tie_idx=tt(tie), noise=tt(noise), action_u=tt(u), temperature=1.0, kernel=kernel, tile=tile)
    if replay:
        kw["replay"] = dict(root_pi=tt(rp["root_pi"]), pi=tt(rp["pi"]), reward=tt(rp["rwd"]), value=tt(rp["value"]))
    else:
        kw["obs"] = tt(obs)
    base = eng.search(S, **kw)
    lo = eng.search(S, out=eng.alloc_search_outputs(B, S, lockstep=True), **kw)
    pl = lo["_plan"]
    for k in ("visits", "root_q", "pi", "action", "sel_steps", "minmax"):
        assert torch.equal(base[k], lo[k]), k
    assert np.array_equal(lo["sel_steps"].cpu().numpy(), ref["sel_steps"])
    g = pl["roots_per_wave"] if pl["wave"] else pl["roots_per_workgroup"]
    ng = -(-B // g)
    lv = lo["lockstep_levels"].cpu().numpy()
    assert (lv[ng:] == 0).all()
    below = np.concatenate([ref["depths"] - 1, np.zeros((ng * g - B, S), np.int32)])
    want = below.reshape(ng, g, S).max(1).sum(1)
    bad = np.flatnonzero(lv[:ng] != want)
    assert bad.size == 0, f"group {bad[0]}: kernel {lv[bad[0]]} levels, oracle {want[bad[0]]} ({bad.size} groups differ)"
    if not replay:
        assert pl == _lib.search_plan(sup, B, S, mzh.search_flags(kernel, tile))
