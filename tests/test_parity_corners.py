"""Parity corners of the search and the env, against fixtures made by
running the reference here (tests/golden/gen_golden.py):

  ucb_np1_vs_np2.npz  child_U (MCTS/node.py:105-123) under the two NumPy promotion rules.  The
                      reference pins numpy==1.25.2 (requirements.txt:17), under which the float32
                      prior times the Python-float w is computed in float64 and rounded once,
                      fl32(fl64(prior) * w); NumPy >= 2 keeps float32, fl32(prior * fl32(w)).  The
                      NumPy-2 column is the reference's own child_U; the NumPy-1 column is the rule
                      evaluated explicitly -- parity unpinned against a NumPy-1 run (no NumPy 1 here).
                      MZH_FLAG_NP1_UCB / oracle np1_ucb select the NumPy-1 rule.
  tie_replay.npz      a run_mcts trace with argmax ties beyond the root's first selection (uniform
                      priors), the reference's np.random.choice replaced by the lowest index in the
                      generator: the kernels resolve such a tie the same way and count it in
                      extra_ties (the reference would have drawn from the RNG: the drop-in warns).
  random_reset.npz    TowersOfHanoi.random_reset (env/hanoi.py:98-109) states from a seeded stream.

Plus the end-to-end agreement of full searches (the oracle's MLP, which the GPU kernels equal bit
for bit) with the reference's own torch-CPU visit counts, pinned at the measured value.
"""
import math
import warnings

import numpy as np
import pytest

from conftest import REPLAY_CASES, golden
from test_oracle_golden import replay_draws, replay_inputs


# ------------------------------------------------------------------------------------- NumPy-1 UCB
def test_ucb_rule_fixture():
    g = golden("ucb_np1_vs_np2.npz")
    prior = g["prior"]
    for npar, nc, p, u1, u2 in zip(g["n_parent"][:2000], g["n_child"][:2000], prior[:2000], g["u_np1"][:2000],
                                   g["u_np2"][:2000]):
        w = (math.log((int(npar) + 19652 + 1) / 19652) + 1.25) * math.sqrt(int(npar)) / (int(nc) + 1)
        assert np.float32(np.float32(p) * np.float32(w)) == u2  # NumPy 2 (NEP 50): float32 arithmetic
        assert np.float32(np.float64(p) * w) == u1  # NumPy 1.25: float64 product, one rounding
    frac = float(g["differ"].mean())
    assert 0.2 < frac < 0.32, frac  # ~26% of evaluations differ in the last bit


def _replay_case(oracle, g, np1):
    n, S = int(g["n"]), int(g["s"])
    noise, tie, u = replay_draws(g)
    return oracle.search(n, S, g["obs"], replay=replay_inputs(g), noise=noise, tie_idx=tie, action_u=u,
                         temperature=float(g["temperature"]), deterministic=bool(g["deterministic"]),
                         discount=float(g["discount"]), np1_ucb=np1)


NP1_CASES = [c for c in REPLAY_CASES if "shared" not in c]


def flip_case():
    """A constructed replay where the two rules pick different children: after the root's first
    selection (child 5, value -5) the two largest priors are adjacent float32 values that NumPy 2
    rounds to the same U (a tie: lowest index, counted as an extra tie) while NumPy 1 separates
    them (child 1 wins).  Found by searching for fl32(p1 * fl32(w)) == fl32(p2 * fl32(w)) with
    fl32(fl64(p1) * w) != fl32(fl64(p2) * w) at N_parent = 1."""
    p1 = np.float32(0.460276335477829)
    p2 = np.nextafter(p1, np.float32(1))
    S = 4
    root_pi = np.array([[p1, p2, 0.02, 0.02, 0.02, 0.02]], np.float32)
    pi = np.full((1, S, 6), 1.0 / 6.0, np.float32)
    value = np.zeros((1, S), np.float32)
    value[0, 0] = -5.0
    obs = np.zeros((1, 9))
    obs[0, [0, 3, 6]] = 1.0
    rp = dict(root_pi=root_pi, pi=pi, rwd=np.zeros((1, S), np.float32), value=value)
    return obs, S, rp, np.array([5], np.int32)


def test_np1_rule_flips_a_choice(oracle):
    obs, S, rp, tie = flip_case()
    o2 = oracle.search(3, S, obs, replay=rp, tie_idx=tie, temperature=1.0, deterministic=True)
    o1 = oracle.search(3, S, obs, replay=rp, tie_idx=tie, temperature=1.0, deterministic=True, np1_ucb=True)
    assert o2["visits"][0, 0] > 0 and o2["visits"][0, 1] == 0  # NumPy 2: the tie resolves to child 0
    assert o1["visits"][0, 1] > 0 and o1["visits"][0, 0] == 0  # NumPy 1: child 1's larger U wins
    assert o2["extra_ties"][0] >= 1 and o1["extra_ties"][0] == o2["extra_ties"][0] - 1


def test_np2_rule_is_the_reference_here(oracle):
    """on every replay fixture the NumPy-2 rule reproduces the reference run (this container's NumPy)"""
    for case in NP1_CASES:
        g = golden(f"replay_{case}.npz")
        assert np.array_equal(_replay_case(oracle, g, False)["visits"], g["visits"])


# ------------------------------------------------------------------------------------- extra ties
def _tie_inputs(g):
    B = g["obs"].shape[0]
    return B, dict(root_pi=g["root_pi"], pi=g["pi"], rwd=g["rwd"], value=g["value"]), np.zeros(B, np.int32)


def test_tie_replay_oracle(oracle):
    g = golden("tie_replay.npz")
    B, rp, tie = _tie_inputs(g)
    o = oracle.search(int(g["n"]), int(g["s"]), g["obs"], replay=rp, tie_idx=tie, temperature=1.0,
                      deterministic=True)
    assert np.array_equal(o["visits"], g["visits"]) and np.array_equal(o["rootQ"], g["rootQ"])
    assert np.array_equal(o["mm_max"], g["mm"][:, 0]) and np.array_equal(o["mm_min"], g["mm"][:, 1])
    assert np.array_equal(o["extra_ties"], g["ties"] - 1) and (o["extra_ties"] > 0).all()


# ------------------------------------------------------------------------------------- random_reset
def test_random_reset_restatement():
    from muzero_hanoi_amd.selfplay import _random_start

    g = golden("random_reset.npz")
    np.random.seed(int(g["seed"]))
    got = [_random_start(int(n), int(gp)) for n, gp in zip(g["n"], g["goal_peg"])]
    assert np.array_equal(got, g["state_idx"])
    assert np.array_equal(np.random.random_sample(4), g["post_rng"])


# ------------------------------------------------------------------------------------- end to end
def _weights(oracle, name):
    from conftest import GOLDEN

    w, in_dim, sup = oracle.load_weights_npz(f"{GOLDEN}/{name}.npz")
    return oracle.flat_weights(w), sup


def test_end_to_end_agreement_with_reference(oracle):
    """Full searches with the restated MLP (k-ordered fp32 FMA chains; the GPU kernels are
    bit-identical to it) against the reference's torch-CPU searches: the MLPs differ in the last
    bits, so a near-tie could flip a histogram.  Measured: every histogram of
    every replay fixture agrees (78 / 78 roots) -- pinned, so a change shows up here."""
    agree = total = 0
    for case in NP1_CASES:
        g = golden(f"replay_{case}.npz")
        n, S, td = int(g["n"]), int(g["s"]), int(g["td"])
        flat, sup = _weights(oracle, f"weights_N{n}_s{int(g['wseed'])}{'' if td else '_mc'}")
        noise, tie, u = replay_draws(g)
        o = oracle.search(n, S, g["obs"], flat=flat, support=sup, noise=noise, tie_idx=tie, action_u=u,
                          temperature=float(g["temperature"]), deterministic=bool(g["deterministic"]),
                          discount=float(g["discount"]))
        same = (o["visits"] == g["visits"]).all(1)
        agree += int(same.sum())
        total += len(same)
    assert (agree, total) == (78, 78)


# ------------------------------------------- end-to-end agreement at scale (part 2)
AGREE = ["n4s50", "n4s200", "n7s100"]


def agree_draws(g):
    """per root r: the reference's global stream re-seeded with seed + r (gen_golden.gen_agreement)"""
    from muzero_hanoi_amd import rng

    ds = []
    for r in range(len(g["obs"])):
        np.random.seed(int(g["seed"]) + r)
        ds.append(rng.predraw(1, deterministic=False, alpha=float(g["alpha"])))
    return tuple(np.concatenate([d[i] for d in ds]) for i in range(3))


def agreement(oracle, case):
    g = golden(f"agree_{case}.npz")
    n, S = int(g["n"]), int(g["s"])
    flat, sup = _weights(oracle, f"weights_N{n}_s{int(g['wseed'])}")
    noise, tie, u = agree_draws(g)
    o = oracle.search(n, S, g["obs"], flat=flat, support=sup, noise=noise, tie_idx=tie, action_u=u,
                      temperature=float(g["temperature"]), discount=float(g["discount"]))
    same = (o["visits"] == g["visits"]).all(1)
    return g, o, same


# measured agreement of the restated MLP's searches with the reference's torch-CPU searches
AGREE_PINNED = {"n4s50": (1024, 1024), "n4s200": (255, 256), "n7s100": (256, 256)}


@pytest.mark.parametrize("case", AGREE)
def test_end_to_end_agreement_at_scale(oracle, case):
    """The reference's run_mcts with its own torch-CPU MuZeroNet on 1,024 / 256 / 256 random roots
    at BASELINE configs' (N, S) shapes vs the oracle's searches (whose MLP the GPU kernels equal bit
    for bit, test_end_to_end_agreement_at_scale_gpu).  The two MLPs differ in the last bits, so a
    root whose root-level UCB decision is a near-tie can flip: the agreement count is pinned and
    every disagreeing root is reported with its smallest root-level UCB gap (fp32)."""
    g, o, same = agreement(oracle, case)
    gaps, deep = g["min_root_gap"], g["min_deep_gap"]
    bad = np.flatnonzero(~same)
    report = [(int(b), float(gaps[b]), float(deep[b]), int(g["zero_gaps"][b]), int(o["extra_ties"][b])) for b in bad]
    print(f"{case}: {int(same.sum())} / {len(same)} histograms equal the reference's; disagreeing roots "
          f"(root, min root-level UCB gap, min deeper gap, exact root ties, oracle extra ties): {report}; "
          f"agreeing roots: median min root-level gap {float(np.median(gaps[same])):.3g}, median min deeper "
          f"gap {float(np.median(deep[same])):.3g}, {int((deep[same] < 1e-6).sum())} with a deeper gap < 1e-6")
    assert (int(same.sum()), len(same)) == AGREE_PINNED[case]


# ------------------------------------------------------------------------------------- GPU
KERNELS = ["coop", "wave16", "wave"]


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("case", AGREE)
def test_end_to_end_agreement_at_scale_gpu(oracle, case, kernel):
    """the kernels' searches on the agreement roots == the oracle's, every root bit for bit (so
    their agreement with the reference is the pinned count of the CPU test above)"""
    import torch

    from muzero_hanoi_amd.engine import Engine

    g, o, same = agreement(oracle, case)
    n, S = int(g["n"]), int(g["s"])
    flat, sup = _weights(oracle, f"weights_N{n}_s{int(g['wseed'])}")
    noise, tie, u = agree_draws(g)
    eng = Engine(n, S, len(g["obs"]), sup)
    eng.load_weights(flat)
    tt = lambda a: torch.tensor(np.asarray(a), device="cuda")
    d = eng.search(S, obs=tt(g["obs"]), tie_idx=tt(tie), noise=tt(noise), action_u=tt(u),
                   temperature=float(g["temperature"]), discount=float(g["discount"]), kernel=kernel)
    for k, ok in (("visits", "visits"), ("root_q", "rootQ"), ("action", "action"), ("sel_steps", "sel_steps")):
        assert np.array_equal(d[k].cpu().numpy(), o[ok]), k
    assert int(((d["visits"].cpu().numpy() == g["visits"]).all(1)).sum()) == AGREE_PINNED[case][0]


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("case", NP1_CASES)
def test_np1_replay_gpu(oracle, case, kernel):
    """MZH_FLAG_NP1_UCB on every kernel == the oracle's NumPy-1 rule, bit for bit"""
    import torch

    from muzero_hanoi_amd.engine import Engine

    g = golden(f"replay_{case}.npz")
    n, S = int(g["n"]), int(g["s"])
    ref = _replay_case(oracle, g, True)
    noise, tie, u = replay_draws(g)
    B = g["obs"].shape[0]
    eng = Engine(n, max(S, 1), B, 33 if int(g["td"]) else 1)
    tt = lambda a: None if a is None else torch.tensor(np.asarray(a), device="cuda")
    rp = replay_inputs(g)
    o = eng.search(S, replay=dict(root_pi=tt(rp["root_pi"]), pi=tt(rp["pi"]), reward=tt(rp["rwd"]),
                                  value=tt(rp["value"])), tie_idx=tt(tie), noise=tt(noise), action_u=tt(u),
                   temperature=float(g["temperature"]), deterministic=bool(g["deterministic"]),
                   discount=float(g["discount"]), np1_ucb=True, kernel=kernel)
    assert np.array_equal(o["visits"].cpu().numpy(), ref["visits"])
    assert np.array_equal(o["root_q"].cpu().numpy(), ref["rootQ"])
    assert np.array_equal(o["minmax"].cpu().numpy()[:, 0], ref["mm_max"])


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", KERNELS)
def test_np1_flip_gpu(oracle, kernel):
    import torch

    from muzero_hanoi_amd.engine import Engine

    obs, S, rp, tie = flip_case()
    eng = Engine(3, S, 1, 33)
    tt = lambda a: torch.tensor(np.asarray(a), device="cuda")
    for np1 in (False, True):
        ref = oracle.search(3, S, obs, replay=rp, tie_idx=tie, temperature=1.0, deterministic=True, np1_ucb=np1)
        o = eng.search(S, replay=dict(root_pi=tt(rp["root_pi"]), pi=tt(rp["pi"]), reward=tt(rp["rwd"]),
                                      value=tt(rp["value"])), tie_idx=tt(tie), temperature=1.0, deterministic=True,
                       np1_ucb=np1, kernel=kernel)
        assert np.array_equal(o["visits"].cpu().numpy(), ref["visits"])
        assert np.array_equal(o["extra_ties"].cpu().numpy(), ref["extra_ties"])


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", KERNELS)
def test_tie_replay_gpu(kernel):
    import torch

    from muzero_hanoi_amd.engine import Engine

    g = golden("tie_replay.npz")
    B, rp, tie = _tie_inputs(g)
    eng = Engine(int(g["n"]), int(g["s"]), B, 33)
    tt = lambda a: torch.tensor(np.asarray(a), device="cuda")
    o = eng.search(int(g["s"]), replay=dict(root_pi=tt(rp["root_pi"]), pi=tt(rp["pi"]), reward=tt(rp["rwd"]),
                                            value=tt(rp["value"])), tie_idx=tt(tie), temperature=1.0,
                   deterministic=True, kernel=kernel)
    assert np.array_equal(o["visits"].cpu().numpy(), g["visits"])
    assert np.array_equal(o["extra_ties"].cpu().numpy(), g["ties"] - 1)


@pytest.mark.gpu
def test_tie_warning_dropin():
    """MCTS.run_mcts tells the caller when a search met an extra tie (its RNG stream then differs
    from the reference's, which would have drawn np.random.choice there)"""
    from muzero_hanoi_amd.mcts import MCTS, RecordedNetwork

    g = golden("tie_replay.npz")
    calls = [dict(root_pi=g["root_pi"][b], pi=g["pi"][b], reward=g["rwd"][b], value=g["value"][b])
             for b in range(g["obs"].shape[0])]
    net = RecordedNetwork(calls, int(g["n"]))
    mcts = MCTS(discount=0.8, root_dirichlet_alpha=0.0, n_simulations=int(g["s"]), batch_s=1, device="cpu")
    np.random.seed(0)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        mcts.run_mcts(g["obs"][0], net, 1.0, True)
    assert mcts.last_extra_ties == int(g["ties"][0]) - 1
    assert any(issubclass(x.category, RuntimeWarning) for x in w)


@pytest.mark.gpu
def test_random_reset_dropin():
    from muzero_hanoi_amd.env import TowersOfHanoi
    from muzero_hanoi_amd.selfplay import state_index

    g = golden("random_reset.npz")
    np.random.seed(int(g["seed"]))
    envs = {}
    for n, gp, want in zip(g["n"], g["goal_peg"], g["state_idx"]):
        env = envs.setdefault((int(n), int(gp)), TowersOfHanoi(N=int(n), max_steps=10, goal_peg=int(gp)))
        obs = env.random_reset()
        assert state_index(env.c_state) == want
        assert obs.sum() == int(n) and obs.dtype == np.float64
    assert np.array_equal(np.random.random_sample(4), g["post_rng"])


@pytest.mark.gpu
@pytest.mark.parametrize("kernel,tile", [("coop", 16), ("coop", 32), ("wave", None), ("wave16", None)])
def test_subnormal_minmax_gap(oracle, kernel, tile):
    """MinMaxStats bounds whose difference is a non-zero subnormal (reachable only from caller-given
    bounds: q values built from fp32 network outputs never get that close) make RN(1/(max - min))
    overflow; the kernels then normalise with the IEEE division (utils_mcts.py:12-16) instead of the
    Markstein quotient, and equal the oracle's exact arithmetic"""
    import torch

    from muzero_hanoi_amd.engine import Engine

    B, S, n = 40, 20, 4
    g = np.random.default_rng(5)
    rp = dict(root_pi=g.dirichlet(np.full(6, 1.0), size=B).astype(np.float32),
              pi=g.dirichlet(np.full(6, 1.0), size=(B, S)).astype(np.float32),
              rwd=np.zeros((B, S), np.float32), value=np.zeros((B, S), np.float32))
    mm = np.tile(np.array([[3e-310, 1e-310]]), (B, 1))
    tie = g.integers(0, 6, B).astype(np.int32)
    obs = np.zeros((B, 3 * n), np.float32)
    ref = oracle.search(n, S, obs, replay=rp, tie_idx=tie, temperature=1.0, deterministic=True, minmax_in=mm)
    assert ref["mm_max"][0] == 3e-310 and ref["mm_min"][0] == 0.0  # the gap stays subnormal
    eng = Engine(n, S, B, 33)
    tt = lambda a: torch.tensor(np.asarray(a), device="cuda")
    o = eng.search(S, replay=dict(root_pi=tt(rp["root_pi"]), pi=tt(rp["pi"]), reward=tt(rp["rwd"]),
                                  value=tt(rp["value"])), tie_idx=tt(tie), minmax_in=tt(mm), temperature=1.0,
                   deterministic=True, kernel=kernel, tile=tile)
    assert np.array_equal(o["visits"].cpu().numpy(), ref["visits"])
    assert np.array_equal(o["root_q"].cpu().numpy(), ref["rootQ"])
    assert np.array_equal(o["minmax"].cpu().numpy()[:, 0], ref["mm_max"])
    assert np.array_equal(o["sel_steps"].cpu().numpy(), ref["sel_steps"])


# ------------------------------- attribution of the one end-to-end disagreement (agree_n4s200 root 210)
# agree_n4s200_trace.npz (gen_golden.gen_agreement_trace): every network call of the reference's
# run_mcts for the roots whose oracle histograms differ from the reference's (root 210) and three
# agreeing controls -- inputs, outputs, logits, the pre-transform scalars (_transform_from_2hot) and
# every torch.sqrt argument / result inside _signed_parabolic (networks.py:152-189).
def _trace_root(oracle, j):
    g, t = golden("agree_n4s200.npz"), golden("agree_n4s200_trace.npz")
    r = int(t["roots"][j])
    flat, sup = _weights(oracle, "weights_N4_s0")
    from muzero_hanoi_amd import rng

    np.random.seed(int(g["seed"]) + r)
    noise, tie, u = rng.predraw(1, deterministic=False, alpha=float(g["alpha"]))
    return g, t, r, flat, noise, tie, u


def _replay_rec(t, j, value=None):
    """the reference's recorded outputs of traced root j as replay records (value optionally swapped)"""
    return dict(root_pi=t["pi"][j][0][None], pi=t["pi"][j][1:][None], rwd=t["rwd"][j][1:][None].astype(np.float32),
                value=(t["v"][j][1:] if value is None else value)[None].astype(np.float32))


def _port_run(oracle, g, r, flat, net):
    """py_port's tree (bit-exact to MCTS/node.py) on one root with the reference's global-stream seeding,
    recording every root-level decision's float32 UCB scores"""
    from oracle import py_port

    rec = []
    orig = py_port.Node.best_child

    def best_child(self, pb_c_base, pb_c_init, discount, mm):
        if self.parent is None:
            q = np.array([mm.normalize(c.rwd + discount * c.Q()) if c.N > 0 else 0 for c in self.children], np.float32)
            u = np.array([c.prior * ((math.log((self.N + pb_c_base + 1) / pb_c_base) + pb_c_init)
                                     * math.sqrt(self.N) / (c.N + 1)) for c in self.children], np.float32)
            rec.append((q + u, [c.W for c in self.children]))
        return orig(self, pb_c_base, pb_c_init, discount, mm)

    py_port.Node.best_child = best_child
    try:
        np.random.seed(int(g["seed"]) + r)
        res = py_port.PortMCTS(float(g["discount"]), float(g["alpha"]), int(g["s"])).run_mcts(
            g["obs"][r].astype(np.float64), net, float(g["temperature"]), False)
    finally:
        py_port.Node.best_child = orig
    return res[3], rec


class _OracleNet:
    """the restated MLP (oracle, bit-equal to the GPU kernels) as a batch-1 network for py_port"""
    num_actions = 6

    def __init__(self, oracle, flat):
        self.o, self.flat, self.calls = oracle, flat, []

    def initial_inference(self, x):
        d = self.o.initial_inference(self.flat, 12, 33, x.numpy()[None].astype(np.float32))
        self.calls.append(d)
        return d["h"][0], 0.0, d["pi"][0], float(d["value"][0])

    def recurrent_inference(self, h, a):
        d = self.o.recurrent_inference(self.flat, 12, 33, h.numpy()[None], np.array([int(a.argmax())]))
        self.calls.append(d)
        return d["h"][0], float(d["reward"][0]), d["pi"][0], float(d["value"][0])


def test_n4s200_disagreement_attribution(oracle):
    """Why root 210 of agree_n4s200 is the one histogram (of 256) the restated MLP's search does not
    reproduce:
      1. the tree is exact: the reference's recorded network outputs replayed through the oracle's
         search give the reference's histogram (the GPU kernels: test_n4s200_trace_replay_gpu);
      2. the first decision that differs is the root-level choice of simulation 54: the reference
         picks child 0 by a float32 UCB margin of 7.2e-5 over child 4, the restated MLP's search
         child 4 -- child 0's summed value W is 2.3e-3 lower on the restated side;
      3. every output before it is equal except the policies (<= 4.5e-8, rounding noise) and ONE
         reward: simulation 4's, one quantum (1.2e-4) of the signed-parabolic output lower.  Its
         cause is the 33-bin expectation: the restated softmax + sum over the REFERENCE's own reward
         logits gives x = -0.0087473392 where torch gave -0.0087471010 (a sum-order / exp difference
         of 2.4e-7 on a cancelling sum), which lands x in the neighbouring output quantum;
         torch.sqrt is correctly rounded at that call;
      4. torch-CPU's not-correctly-rounded sqrt is not the cause: at the one value call where it is
         1 ulp off (simulation 128, after the divergence), substituting the correctly rounded
         result leaves the reference's histogram unchanged.
    The three control roots agree and reach the same histogram by every route."""
    g, t, r, flat, noise, tie, u = _trace_root(oracle, 0)
    assert r == 210 and int(t["n_bad"]) == 1
    kw = dict(noise=noise, tie_idx=tie, action_u=u, temperature=1.0, discount=0.8)
    obs = g["obs"][r][None]
    # 1. tree exactness
    o = oracle.search(4, 200, obs, replay=_replay_rec(t, 0), **kw)
    assert np.array_equal(o["visits"][0], g["visits"][r])
    e2e = oracle.search(4, 200, obs, flat=flat, support=33, **kw)["visits"][0]
    assert not np.array_equal(e2e, g["visits"][r])
    # 2. first diverging decision (py_port tree, reference outputs vs the restated MLP)
    from oracle import py_port

    vis_ref, dec_ref = _port_run(oracle, g, r, flat, py_port.ReplayNet(t["pi"][0][0], t["pi"][0][1:],
                                                                    t["rwd"][0][1:], t["v"][0][1:]))
    onet = _OracleNet(oracle, flat)
    vis_orc, dec_orc = _port_run(oracle, g, r, flat, onet)
    assert np.array_equal(vis_ref, g["visits"][r]) and np.array_equal(vis_orc, e2e)
    picks = [(int(np.argmax(a[0])), int(np.argmax(b[0]))) for a, b in zip(dec_ref, dec_orc)]
    first = next(i for i, (a, b) in enumerate(picks) if a != b)
    assert first == 53 and picks[first] == (0, 4)  # decision of simulation 54
    s_ref, s_orc = dec_ref[first][0], dec_orc[first][0]
    gap_ref, gap_orc = float(s_ref[0]) - float(s_ref[4]), float(s_orc[0]) - float(s_orc[4])
    dW0 = dec_orc[first][1][0] - dec_ref[first][1][0]
    print(f"simulation 54: reference UCB(child 0) - UCB(child 4) = {gap_ref:.3g}, restated {gap_orc:.3g}; "
          f"child 0 W differs by {dW0:.3g}")
    assert 0 < gap_ref < 1e-4 and gap_orc < 0 and -3e-3 < dW0 < -2e-3
    # 3. what differs before it
    oc = onet.calls[:54]
    val = np.array([float(c["value"][0]) for c in oc], np.float32)
    rwd = np.array([float(c["reward"][0]) for c in oc], np.float32)
    pi = np.array([c["pi"][0] for c in oc], np.float32)
    assert np.array_equal(val, t["v"][0][:54].astype(np.float32))
    assert float(np.abs(pi - t["pi"][0][:54]).max()) < 1e-7
    drw = np.flatnonzero(rwd[1:] != t["rwd"][0][1:54].astype(np.float32)) + 1
    assert list(drw) == [4]
    assert -1.3e-4 < float(rwd[4]) - float(t["rwd"][0][4]) < -1.1e-4
    x_restated = np.float32(oracle.logits_expectation(t["rl"][0][4]))
    x_torch = t["xr"][0][4]
    print(f"simulation 4 reward: x from the reference's logits restated {x_restated!r}, torch {x_torch!r}")
    assert x_restated != x_torch and abs(float(x_restated) - float(x_torch)) < 1e-6
    assert np.float32(oracle.signed_parabolic(x_torch)) == np.float32(t["rwd"][0][4])
    assert np.float32(oracle.signed_parabolic(x_restated)) == rwd[4]
    sq = t["sqrt_r"][0][4]
    assert np.sqrt(np.float32(sq[0])) == sq[1]  # torch's sqrt exact at that call
    # 4. torch sqrt's 1-ulp misses: swapping in the correctly rounded value changes nothing
    sv = t["sqrt_v"][0][1:]
    miss = np.flatnonzero(np.sqrt(sv[:, 0].astype(np.float32)) != sv[:, 1])
    assert list(miss + 1) == [128]
    fixed = t["v"][0][1:].copy()
    fixed[miss] = [oracle.signed_parabolic(x) for x in t["xv"][0][1:][miss]]
    assert np.float32(fixed[miss][0]) != np.float32(t["v"][0][1:][miss][0])
    o = oracle.search(4, 200, obs, replay=_replay_rec(t, 0, value=fixed), **kw)
    assert np.array_equal(o["visits"][0], g["visits"][r])
    # controls
    for j in range(1, len(t["roots"])):
        g, t, rc, flat, noise, tie, u = _trace_root(oracle, j)
        kwc = dict(noise=noise, tie_idx=tie, action_u=u, temperature=1.0, discount=0.8)
        o = oracle.search(4, 200, g["obs"][rc][None], replay=_replay_rec(t, j), **kwc)
        assert np.array_equal(o["visits"][0], g["visits"][rc])


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", KERNELS)
def test_n4s200_trace_replay_gpu(oracle, kernel):
    """the traced roots (root 210 and the controls) with the reference's own recorded outputs
    replayed through every kernel: the reference's histograms, bit for bit"""
    import torch

    from muzero_hanoi_amd.engine import Engine

    t = golden("agree_n4s200_trace.npz")
    J = len(t["roots"])
    parts = [_trace_root(oracle, j) for j in range(J)]
    g = parts[0][0]
    noise = np.concatenate([p[4] for p in parts]); tie = np.concatenate([p[5] for p in parts])
    u = np.concatenate([p[6] for p in parts])
    rp = dict(root_pi=t["pi"][:, 0], pi=t["pi"][:, 1:], reward=t["rwd"][:, 1:].astype(np.float32),
              value=t["v"][:, 1:].astype(np.float32))
    eng = Engine(4, 200, J, 33)
    tt = lambda a: torch.tensor(np.asarray(a), device="cuda")
    o = eng.search(200, replay={k: tt(v) for k, v in rp.items()}, tie_idx=tt(tie), noise=tt(noise), action_u=tt(u),
                   temperature=1.0, discount=0.8, kernel=kernel)
    assert np.array_equal(o["visits"].cpu().numpy(), g["visits"][t["roots"]])
