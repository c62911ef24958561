"""Generate the golden fixtures under tests/golden/ from the reference itself.

Runs ONLY in the build container (the reference is not present on the GPU box).
It imports A-Andrews/Muzero-Hanoi from /root/reference with a one-line `seaborn` stub
(seaborn is imported at module top by reference utils.py:5 but only used for plotting),
never writes into the reference tree (PYTHONDONTWRITEBYTECODE), and saves small .npz/.json
files of INPUTS and OUTPUTS only -- no reference source travels with them.

    python tests/golden/gen_golden.py            # regenerate every fixture

Fixtures (see tests/golden/README.md):
  env_N{3,4,7}.npz        every state x action through TowersOfHanoi.step (env/hanoi.py:47-84)
  env_maxsteps.npz        step-counter / goal quirk sequences (env/hanoi.py:65-80)
  solver_N{3,4,7}.npz     hanoi_solver for all 3^N states (env/hanoi_utils.py:4-26)
  weights_N{N}_s{seed}.npz  MuZeroNet(TD_return=...) state_dict after torch.manual_seed(seed)
  mlp_N{N}_s{seed}.npz    initial/recurrent inference I/O + raw logits (networks.py:71-150)
  replay_<case>.npz       full run_mcts traces: every network call's inputs/outputs, RNG events,
                          final visits / pi / rootQ / action / min-max (MCTS/mcts.py:34-126)
  training_<case>.npz     Buffer sampling + Muzero._update steps: indices, IS weights, losses,
                          new priorities, parameters and Adam moments (Muzero.py:209-274, buffer.py)
  acting_<case>.npz       acting_ablations.get_results runs (every network output, actions, env
                          results, MinMaxStats, the returned data, the RNG position after)
  illegal_<case>.npz      illegal_move_rate_comparison.illegal_move_rate runs (same records)
  ucb_np1_vs_np2.npz      child_U under NumPy-2 (the reference's own, here) and NumPy-1 promotion
  tie_replay.npz          a run_mcts trace with argmax ties beyond the root's first selection
  random_reset.npz        TowersOfHanoi.random_reset start states from a seeded global stream
  play_policy.npz         generate_play_policy over random histograms at non-integer exponents
  bad_temperature.npz     run_mcts with invalid temperatures between valid ones (state after the raise)
  agree_<case>.npz        the reference's run_mcts (torch-CPU network) on 256-1024 roots per
                          (N, S) shape: visit histograms + root-level UCB gaps (near-tie report)
  agree_n4s200_trace.npz  every network call (I/O, logits, pre-transform scalars, torch.sqrt
                          arguments/results) of the roots the restated MLP's search disagrees on
"""
import json
import os
import sys
import types

sys.dont_write_bytecode = True
os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

sys.modules.setdefault("seaborn", types.ModuleType("seaborn"))
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from env.hanoi import TowersOfHanoi  # noqa: E402
from env.hanoi_utils import hanoi_solver  # noqa: E402
from MCTS.mcts import MCTS  # noqa: E402
from networks import MuZeroNet  # noqa: E402

torch.set_num_threads(1)

WEIGHT_KEYS = [
    f"{net}.{layer}.{kind}"
    for net in ("representation_net", "dynamic_net", "rwd_net", "policy_net", "value_net")
    for layer in (0, 2)
    for kind in ("weight", "bias")
]


def state_index(state, n):
    idx = 0
    for s in state:
        idx = idx * 3 + int(s)
    return idx


# --------------------------------------------------------------------------- env
def gen_env(n):
    env = TowersOfHanoi(N=n, max_steps=10**9)
    ns = len(env.states)
    nxt = np.zeros((ns, 6), np.int32)  # env.c_state index after the step
    moved = np.zeros((ns, 6), np.int32)  # state encoded in the returned one-hot
    rwd = np.zeros((ns, 6), np.float64)
    done = np.zeros((ns, 6), np.uint8)
    illegal = np.zeros((ns, 6), np.uint8)
    legal = np.zeros((ns, 6), np.uint8)
    for i, st in enumerate(env.states):
        for a in range(6):
            env.reset()
            env.c_state = st
            env.step_counter = 0
            legal[i, a] = env._move_allowed(env.moves[a])
            obs, r, d, ill = env.step(a)
            onehot = obs.reshape(n, 3)
            assert onehot.sum() == n
            moved[i, a] = state_index(onehot.argmax(1), n)
            nxt[i, a] = state_index(env.c_state, n)
            rwd[i, a] = r
            done[i, a] = d
            illegal[i, a] = ill
    np.savez_compressed(
        os.path.join(HERE, f"env_N{n}.npz"),
        n=n, next_state=nxt, moved_state=moved, reward=rwd, done=done, illegal=illegal,
        legal=legal, goal=state_index(env.goal, n), n_states=ns,
        moves=np.array(env.moves, np.int32),
    )


def gen_env_maxsteps():
    """Sequences exercising step_counter / max_steps / goal-reset (env/hanoi.py:65-80)."""
    rows = []
    rng = np.random.RandomState(7)
    for n, max_steps, init_idx in [(3, 5, 0), (3, 200, 0), (4, 7, 5), (3, 3, 25)]:
        env = TowersOfHanoi(N=n, max_steps=max_steps, init_state_idx=init_idx)
        env.reset()
        for t in range(3 * max_steps if max_steps < 50 else 60):
            if not env.reset_check:
                env.reset()
            a = int(rng.randint(6))
            before = state_index(env.c_state, n)
            ctr_before = env.step_counter
            obs, r, d, ill = env.step(a)
            rows.append((n, max_steps, init_idx, before, ctr_before, a,
                         state_index(obs.reshape(n, 3).argmax(1), n),
                         state_index(env.c_state, n), float(r), int(d), int(ill),
                         env.step_counter, int(env.reset_check)))
    # an optimal solve that reaches the goal: c_state must NOT advance on the goal step
    env = TowersOfHanoi(N=3, max_steps=200, init_state_idx=state_index((1, 2, 2), 3))
    env.reset()
    before = state_index(env.c_state, 3)
    a = env.moves.index((1, 2))
    obs, r, d, ill = env.step(a)
    rows.append((3, 200, env.init_state_idx, before, 0, a,
                 state_index(obs.reshape(3, 3).argmax(1), 3), state_index(env.c_state, 3),
                 float(r), int(d), int(ill), env.step_counter, int(env.reset_check)))
    arr = np.array(rows, dtype=np.float64)
    np.savez_compressed(
        os.path.join(HERE, "env_maxsteps.npz"), rows=arr,
        columns=np.array(["n", "max_steps", "init_idx", "state_before", "ctr_before", "action",
                          "moved_state", "c_state_after", "reward", "done", "illegal",
                          "ctr_after", "reset_check_after"]),
    )


def gen_solver(n):
    env = TowersOfHanoi(N=n, max_steps=1)
    vals = np.array([hanoi_solver(tuple(s)) for s in env.states], np.int32)
    vals_g0 = np.array([hanoi_solver(tuple(s), 0) for s in env.states], np.int32)
    np.savez_compressed(os.path.join(HERE, f"solver_N{n}.npz"), n=n, moves=vals, moves_goal0=vals_g0)


# --------------------------------------------------------------------------- network
def make_net(n, seed, td=True):
    torch.manual_seed(seed)
    return MuZeroNet(rpr_input_s=3 * n, action_s=6, lr=0.002, device="cpu", TD_return=td)


def save_weights(net, n, seed, td=True):
    sd = net.state_dict()
    path = os.path.join(HERE, f"weights_N{n}_s{seed}{'' if td else '_mc'}.npz")
    np.savez_compressed(path, **{k: sd[k].numpy() for k in WEIGHT_KEYS})


def gen_mlp(n, seed, td=True, batch=24):
    net = make_net(n, seed, td)
    save_weights(net, n, seed, td)
    rng = np.random.RandomState(1000 + seed + n)
    # observations: one-hot Hanoi states + a few arbitrary float vectors (noise-injection style)
    states = rng.randint(0, 3, size=(batch, n))
    x = np.zeros((batch, 3 * n), np.float32)
    for b in range(batch):
        x[b, np.arange(n) * 3 + states[b]] = 1.0
    x[-4:] = rng.uniform(-1, 1, size=(4, 3 * n)).astype(np.float32)
    h_in = rng.uniform(0, 1, size=(batch, 64)).astype(np.float32)
    a_in = rng.randint(0, 6, size=batch).astype(np.int64)

    ii_h, ii_r, ii_pi, ii_v = [], [], [], []
    ri_h, ri_r, ri_pi, ri_v = [], [], [], []
    pol_logits0, val_logits0 = [], []
    pol_logits1, val_logits1, rwd_logits1, hraw1 = [], [], [], []
    with torch.no_grad():
        for b in range(batch):
            xt = torch.from_numpy(x[b])
            h, r, pi, v = net.initial_inference(xt)
            ii_h.append(h); ii_r.append(r); ii_pi.append(pi); ii_v.append(v)
            hs = net.represent(xt)
            pol_logits0.append(net.policy_net(hs).numpy())
            val_logits0.append(net.value_net(hs).numpy())

            ht = torch.from_numpy(h_in[b])
            at = torch.nn.functional.one_hot(torch.tensor([a_in[b]]), 6).squeeze().float()
            h2, r2, pi2, v2 = net.recurrent_inference(ht, at)
            ri_h.append(h2); ri_r.append(r2); ri_pi.append(pi2); ri_v.append(v2)
            hr = net.dynamic_net(torch.cat([ht, at], -1))
            hraw1.append(hr.numpy())
            rwd_logits1.append(net.rwd_net(hr).numpy())
            hn = net.normalize_h_state(hr)
            pol_logits1.append(net.policy_net(hn).numpy())
            val_logits1.append(net.value_net(hn).numpy())
    np.savez_compressed(
        os.path.join(HERE, f"mlp_N{n}_s{seed}{'' if td else '_mc'}.npz"),
        n=n, seed=seed, td=int(td), x=x, h_in=h_in, a_in=a_in,
        ii_h=np.array(ii_h, np.float32), ii_rwd=np.array(ii_r, np.float64),
        ii_pi=np.array(ii_pi, np.float32), ii_value=np.array(ii_v, np.float64),
        ii_policy_logits=np.array(pol_logits0, np.float32),
        ii_value_logits=np.array(val_logits0, np.float32),
        ri_h=np.array(ri_h, np.float32), ri_rwd=np.array(ri_r, np.float64),
        ri_pi=np.array(ri_pi, np.float32), ri_value=np.array(ri_v, np.float64),
        ri_h_raw=np.array(hraw1, np.float32), ri_rwd_logits=np.array(rwd_logits1, np.float32),
        ri_policy_logits=np.array(pol_logits1, np.float32),
        ri_value_logits=np.array(val_logits1, np.float32),
    )


# --------------------------------------------------------------------------- search traces
class Recorder:
    """Duck-typed network (MCTS/mcts.py:50,96,102): calls the real MuZeroNet, records I/O."""

    def __init__(self, net):
        self.net = net
        self.num_actions = net.num_actions
        self.calls = []

    def initial_inference(self, x):
        out = self.net.initial_inference(x)
        self.calls.append(("i", x.numpy().copy(), -1, out))
        return out

    def recurrent_inference(self, h, a):
        out = self.net.recurrent_inference(h, a)
        self.calls.append(("r", h.numpy().copy(), int(a.argmax()), out))
        return out


class TracingMCTS(MCTS):
    """Subclass (in this script only) that captures the root visit histogram and the
    Dirichlet-mixed priors; the reference files are not modified."""

    def generate_play_policy(self, visits_count, temperature):
        self.last_visits = np.asarray(visits_count).copy()
        return super().generate_play_policy(visits_count, temperature)

    def add_dirichlet_noise(self, prob, eps=0.25, alpha=0.25):
        out = super().add_dirichlet_noise(prob, eps=eps, alpha=alpha)
        self.last_noised = np.asarray(out, np.float64).copy()
        return out


def gen_replay(name, n, s, n_roots, deterministic, alpha, temperature, seed=1, wseed=0,
               shared=False, td=True, discount=0.8):
    net = make_net(n, wseed, td)
    np.random.seed(seed)
    rec_choice = []
    orig_choice = np.random.choice

    def choice(a, *args, **kw):
        r = orig_choice(a, *args, **kw)
        size = a if isinstance(a, (int, np.integer)) else len(a)
        rec_choice.append((len(rec_per_root) - 1, size, "p" in kw, int(r)))
        return r

    np.random.choice = choice
    env = TowersOfHanoi(N=n, max_steps=200)
    goal = state_index(env.goal, n)
    rs = np.random.RandomState(seed + 17)  # root states (separate stream: not the global RNG)
    root_idx = []
    while len(root_idx) < n_roots:
        i = int(rs.randint(3 ** n))
        if i != goal:
            root_idx.append(i)
    rec_per_root = []
    out = dict(visits=[], pi=[], rootQ=[], action=[], mm_max=[], mm_min=[], noised=[],
               latent=[], calls_h=[], calls_a=[], out_h=[], out_rwd=[], out_pi=[], out_v=[],
               obs=[])
    mcts = None
    try:
        for r, idx in enumerate(root_idx):
            rec_per_root.append(r)
            if mcts is None or not shared:
                mcts = TracingMCTS(discount=discount, root_dirichlet_alpha=alpha,
                                   n_simulations=s, batch_s=256, device="cpu")
            mcts.last_noised = None
            st = env.states[idx]
            obs = np.zeros(3 * n)
            obs[np.arange(n) * 3 + np.array(st)] = 1.0
            recorder = Recorder(net)
            action, pi, q = mcts.run_mcts(obs, recorder, temperature, deterministic)
            out["visits"].append(mcts.last_visits.astype(np.int32))
            out["pi"].append(np.asarray(pi, np.float64))
            out["rootQ"].append(float(q))
            out["action"].append(int(action))
            out["mm_max"].append(float(mcts.min_max_stats.maximum))
            out["mm_min"].append(float(mcts.min_max_stats.minimum))
            out["noised"].append(mcts.last_noised if mcts.last_noised is not None
                                 else np.full(6, np.nan))
            lat = [int(t.item()) for t in mcts.return_latent_actions()]
            out["latent"].append(lat + [-1] * (s + 2 - len(lat)))
            out["obs"].append(obs)
            calls = recorder.calls
            assert calls[0][0] == "i" and len(calls) == s + 1
            out["calls_h"].append(np.array([c[1] if c[0] == "r" else np.zeros(64, np.float32)
                                            for c in calls], np.float32))
            out["calls_a"].append(np.array([c[2] for c in calls], np.int32))
            out["out_h"].append(np.array([c[3][0] for c in calls], np.float32))
            out["out_rwd"].append(np.array([c[3][1] for c in calls], np.float64))
            out["out_pi"].append(np.array([c[3][2] for c in calls], np.float32))
            out["out_v"].append(np.array([c[3][3] for c in calls], np.float64))
    finally:
        np.random.choice = orig_choice
    ch = np.array(rec_choice, np.int64).reshape(-1, 4)
    np.savez_compressed(
        os.path.join(HERE, f"replay_{name}.npz"),
        n=n, s=s, seed=seed, wseed=wseed, td=int(td), deterministic=int(deterministic),
        alpha=alpha, temperature=temperature, shared=int(shared), discount=discount,
        root_idx=np.array(root_idx, np.int32), obs=np.array(out["obs"], np.float64),
        visits=np.array(out["visits"]), pi=np.array(out["pi"]),
        rootQ=np.array(out["rootQ"]), action=np.array(out["action"], np.int32),
        mm_max=np.array(out["mm_max"]), mm_min=np.array(out["mm_min"]),
        noised=np.array(out["noised"], np.float64), latent=np.array(out["latent"], np.int32),
        calls_h=np.array(out["calls_h"]), calls_a=np.array(out["calls_a"]),
        out_h=np.array(out["out_h"]), out_rwd=np.array(out["out_rwd"]),
        out_pi=np.array(out["out_pi"]), out_v=np.array(out["out_v"]),
        choice_events=ch,  # (root, n_candidates, has_p, result)
    )
    return ch


REPLAY_CASES = [
    # name, n, s, roots, deterministic, alpha, T, extra
    ("n3s25_det", 3, 25, 8, True, 0.0, 1.0, {}),
    ("n3s25_sto", 3, 25, 8, False, 0.25, 1.0, {}),
    ("n4s50_sto", 4, 50, 8, False, 0.25, 1.0, {}),
    ("n4s50_det_t0", 4, 50, 6, True, 0.25, 0.0, {}),
    ("n4s50_sto_t05", 4, 50, 6, False, 0.25, 0.5, {}),
    ("n4s50_sto_t01", 4, 50, 4, False, 0.25, 0.1, {}),
    ("n4s50_alpha03", 4, 50, 4, False, 0.3, 1.0, {}),
    ("n4s50_shared", 4, 50, 6, False, 0.25, 1.0, {"shared": True}),
    ("n4s200_sto", 4, 200, 3, False, 0.25, 1.0, {}),
    ("n7s100_sto", 7, 100, 3, False, 0.25, 1.0, {}),
    ("n3s25_mc", 3, 25, 4, False, 0.25, 1.0, {"td": False}),
    ("n4s1_sto", 4, 1, 4, False, 0.25, 1.0, {}),
    # non-integer play-policy exponents (np.power with 1/T = 3.33.., 1.43.., 1.11..; mcts.py:173-174)
    ("n4s50_sto_t03", 4, 50, 6, False, 0.25, 0.3, {}),
    ("n4s50_sto_t07", 4, 50, 6, False, 0.25, 0.7, {}),
    ("n3s25_sto_t09", 3, 25, 8, False, 0.25, 0.9, {}),
]


def gen_play_policy(n_hist=600, seed=71):
    """MCTS.generate_play_policy (mcts.py:154-176) of the reference over random visit histograms
    (sums S in {1, 25, 50, 100, 200}, zeros included) at temperatures with non-integer exponents
    (and a few integer ones): the NumPy np.power values the play policy is built from."""
    m = MCTS(discount=0.8, root_dirichlet_alpha=0.25, n_simulations=1, batch_s=1, device="cpu")
    rs = np.random.RandomState(seed)
    temps = np.array([0.3, 0.7, 0.9, 0.35, 0.45, 0.6, 0.8, 0.95, 0.999, 0.21, 1.0, 0.5, 0.25], np.float64)
    hist, sums = [], []
    for i in range(n_hist):
        S = [1, 25, 50, 100, 200][i % 5]
        k = rs.randint(1, 7)  # children with visits
        p = rs.dirichlet(np.full(k, 0.5))
        v = np.zeros(6, np.int64)
        v[rs.choice(6, k, replace=False)] = rs.multinomial(S, p)
        hist.append(v)
        sums.append(S)
    hist = np.array(hist, np.int64)
    pi = np.array([[m.generate_play_policy(h, float(t)) for h in hist] for t in temps], np.float64)
    # the raw powers too, elementwise over 0..200 (the table a device pow must reproduce)
    powers = np.array([np.power(np.arange(201, dtype=np.int64), max(1.0, min(5.0, 1.0 / float(t))))
                       for t in temps], np.float64)
    np.savez_compressed(os.path.join(HERE, "play_policy.npz"), temps=temps, visits=hist.astype(np.int32),
                        sums=np.array(sums, np.int32), pi=pi, powers=powers)


def gen_agreement(name, n, s, n_roots, seed, wseed=0, alpha=0.25, temperature=1.0, discount=0.8):
    """End to end at scale (hard part 2): the reference's own run_mcts with its
    torch-CPU MuZeroNet on n_roots random non-goal roots, the global NumPy stream re-seeded with
    seed + r before root r (so every root's draws are reproducible on their own).  Per root the
    visit histogram, and the gap between the largest and second-largest float32 UCB score
    (node.py:83-88): its minimum over the root-level decisions and over the deeper ones of visited
    nodes -- the near-tie diagnostic for roots whose histograms an ulp-level MLP difference could
    flip."""
    from MCTS.node import Node

    net = make_net(n, wseed, True)
    env = TowersOfHanoi(N=n, max_steps=200)
    goal = state_index(env.goal, n)
    rs = np.random.RandomState(seed + 17)
    root_idx = []
    while len(root_idx) < n_roots:
        i = int(rs.randint(3 ** n))
        if i != goal:
            root_idx.append(i)
    margins, deep = [], []
    orig = Node.best_child

    def best_child(self, config, min_max_stats):
        u = self.child_Q(config, min_max_stats) + self.child_U(config)
        srt = np.sort(u)
        gap = float(srt[-1] - srt[-2])
        if self.parent is None:  # a root-level decision
            margins[-1].append(gap)
        elif self.N > 0:  # a deeper decision (N = 0: the uniform-prior tie of a fresh node)
            deep[-1] = min(deep[-1], gap)
        return orig(self, config, min_max_stats)

    Node.best_child = best_child
    visits, obs_all, min_gap, n_zero = [], [], [], []
    try:
        for r, idx in enumerate(root_idx):
            np.random.seed(seed + r)
            margins.append([])
            deep.append(np.inf)
            mcts = TracingMCTS(discount=discount, root_dirichlet_alpha=alpha, n_simulations=s, batch_s=256,
                               device="cpu")
            obs = np.zeros(3 * n)
            obs[np.arange(n) * 3 + np.array(env.states[idx])] = 1.0
            with torch.no_grad():
                mcts.run_mcts(obs, net, temperature, False)
            visits.append(mcts.last_visits.astype(np.int32))
            obs_all.append(obs)
            gaps = np.array(margins[-1][1:])  # the first decision is the 6-way tie at N_root = 0
            min_gap.append(float(gaps.min()) if gaps.size else np.inf)
            n_zero.append(int((gaps == 0).sum()))
    finally:
        Node.best_child = orig
    np.savez_compressed(os.path.join(HERE, f"agree_{name}.npz"), n=n, s=s, seed=seed, wseed=wseed, alpha=alpha,
                        temperature=temperature, discount=discount, root_idx=np.array(root_idx, np.int32),
                        obs=np.array(obs_all, np.float32), visits=np.array(visits, np.int32),
                        min_root_gap=np.array(min_gap, np.float64), zero_gaps=np.array(n_zero, np.int32),
                        min_deep_gap=np.array(deep, np.float64))


def gen_agreement_trace(name, n, s, n_roots, seed, wseed=0, alpha=0.25, temperature=1.0, discount=0.8,
                        controls=3):
    """Every network call of the reference's run_mcts (torch-CPU MuZeroNet) for the roots of agree_<name>
    whose visit histograms the oracle's search does not reproduce, plus `controls` agreeing roots:
    inputs (parent latent, action), outputs (latent, reward, pi, value), the raw logits (policy 6,
    value / reward 33, by forward hooks on the reference's own heads), the pre-transform scalars
    (_transform_from_2hot) and every torch.sqrt argument / result inside _signed_parabolic
    (networks.py:186-189) -- so the first simulation where the restated MLP leaves the reference, and
    which operation moved it, can be read off (tests/test_parity_corners.py).  Same seeds and roots as
    gen_agreement."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import oracle as orc

    g = np.load(os.path.join(HERE, f"agree_{name}.npz"))
    w = {k: v for k, v in np.load(os.path.join(HERE, f"weights_N{n}_s{wseed}.npz")).items()}
    flat = orc.flat_weights(w)
    B = len(g["obs"])
    noise, tie, u = [], [], []
    for r in range(B):
        np.random.seed(seed + r)
        noise.append(np.random.dirichlet(np.ones(6, np.float32) * alpha))
        tie.append(np.random.choice(np.arange(6)))
        u.append(np.random.random_sample())
    o = orc.search(n, s, g["obs"], flat=flat, support=33, noise=np.array(noise), tie_idx=np.array(tie),
                   action_u=np.array(u), temperature=temperature, discount=discount)
    bad = np.flatnonzero(~(o["visits"] == g["visits"]).all(1))
    good = np.flatnonzero((o["visits"] == g["visits"]).all(1))[:controls]
    roots = np.concatenate([bad, good]).astype(np.int32)

    net = make_net(n, wseed, True)
    cap = {}
    hooks = [getattr(net, m).register_forward_hook(lambda mod, i, out, m=m: cap.setdefault(m, out.detach().clone()))
             for m in ("policy_net", "value_net", "rwd_net")]
    orig_t2h = net._transform_from_2hot

    def t2h(probs, lo, hi):
        x = orig_t2h(probs, lo, hi)
        cap.setdefault("x", []).append(float(x.reshape(-1)[0]))
        return x

    net._transform_from_2hot = t2h
    orig_sqrt = torch.sqrt

    def sqrt(t, *a, **k):
        r = orig_sqrt(t, *a, **k)
        cap.setdefault("sqrt", []).append((float(t.reshape(-1)[0]), float(r.reshape(-1)[0])))
        return r

    recs = []

    class Rec:
        num_actions = net.num_actions

        def _call(self, kind, fn, h, a):
            cap.clear()
            out = fn()
            xs, sq = cap.get("x", []), cap.get("sqrt", [])
            # recurrent: reward then value (dynamics before prediction, networks.py:104-107)
            xr, xv = (xs[0], xs[1]) if kind == "r" else (0.0, xs[0])
            sr, sv = (sq[0], sq[1]) if kind == "r" else ((0.0, 0.0), sq[0])
            recs[-1].append(dict(
                kind=kind, h_in=h, a=a, h=np.asarray(out[0], np.float32), rwd=float(out[1]),
                pi=np.asarray(out[2], np.float32), v=float(out[3]),
                pl=cap["policy_net"].numpy().reshape(-1), vl=cap["value_net"].numpy().reshape(-1),
                rl=cap["rwd_net"].numpy().reshape(-1) if kind == "r" else np.zeros(33, np.float32),
                xv=xv, xr=xr, sqrt_v=sv, sqrt_r=sr))
            return out

        def initial_inference(self, x):
            return self._call("i", lambda: net.initial_inference(x), np.zeros(64, np.float32), -1)

        def recurrent_inference(self, h, a):
            return self._call("r", lambda: net.recurrent_inference(h, a), h.numpy().reshape(-1).copy(),
                              int(a.argmax()))

    torch.sqrt = sqrt
    try:
        for r in roots:
            recs.append([])
            np.random.seed(seed + int(r))
            mcts = TracingMCTS(discount=discount, root_dirichlet_alpha=alpha, n_simulations=s, batch_s=256,
                               device="cpu")
            mcts.run_mcts(g["obs"][r].astype(np.float64), Rec(), temperature, False)
            assert np.array_equal(mcts.last_visits, g["visits"][r]), "re-run differs from agree fixture"
    finally:
        torch.sqrt = orig_sqrt
        for hk in hooks:
            hk.remove()
    st = lambda k, dt: np.array([[c[k] for c in rr] for rr in recs], dt)
    np.savez_compressed(
        os.path.join(HERE, f"agree_{name}_trace.npz"), n=n, s=s, seed=seed, roots=roots, n_bad=len(bad),
        h_in=st("h_in", np.float32), a=st("a", np.int32), h=st("h", np.float32), rwd=st("rwd", np.float64),
        pi=st("pi", np.float32), v=st("v", np.float64), pl=st("pl", np.float32), vl=st("vl", np.float32),
        rl=st("rl", np.float32), xv=st("xv", np.float32), xr=st("xr", np.float32),
        sqrt_v=st("sqrt_v", np.float32), sqrt_r=st("sqrt_r", np.float32))
    return roots, len(bad)


def gen_bad_temperature(n=3, s=25, seed=81, wseed=0):
    """run_mcts calls on one MCTS instance with an invalid temperature between valid ones: the
    reference runs the whole search (Dirichlet and tie draws, MinMaxStats, latent_actions) and
    raises in generate_play_policy (mcts.py:113,163-166) before its action draw (mcts.py:120)."""
    net = make_net(n, wseed, True)
    env = TowersOfHanoi(N=n, max_steps=200)
    temps = [1.5, 1.0, -0.1, 0.5]
    roots = [3, 11, 7, 20]
    np.random.seed(seed)
    mcts = TracingMCTS(discount=0.8, root_dirichlet_alpha=0.25, n_simulations=s, batch_s=256, device="cpu")
    rec = dict(obs=[], raised=[], action=[], pi=[], mm_max=[], mm_min=[], latent=[], out_pi=[], out_rwd=[],
               out_v=[])
    for t, idx in zip(temps, roots):
        obs = np.zeros(3 * n)
        obs[np.arange(n) * 3 + np.array(env.states[idx])] = 1.0
        recorder = Recorder(net)
        raised, action, pi = 0, -1, np.full(6, np.nan)
        try:
            action, pi, _ = mcts.run_mcts(obs, recorder, t, False)
        except ValueError:
            raised = 1
        rec["obs"].append(obs)
        rec["raised"].append(raised)
        rec["action"].append(int(action))
        rec["pi"].append(np.asarray(pi, np.float64))
        rec["mm_max"].append(float(mcts.min_max_stats.maximum))
        rec["mm_min"].append(float(mcts.min_max_stats.minimum))
        lat = [int(x.item()) for x in mcts.return_latent_actions()]
        rec["latent"].append(lat + [-1] * (s + 2 - len(lat)))
        rec["out_pi"].append(np.array([c[3][2] for c in recorder.calls], np.float32))
        rec["out_rwd"].append(np.array([c[3][1] for c in recorder.calls], np.float64))
        rec["out_v"].append(np.array([c[3][3] for c in recorder.calls], np.float64))
    post = np.random.random_sample(4)
    np.savez_compressed(os.path.join(HERE, "bad_temperature.npz"), n=n, s=s, seed=seed, temps=np.array(temps),
                        post_rng=post, **{k: np.array(v) for k, v in rec.items()})


AGREE_CASES = [
    # name, n, s, roots, seed: BASELINE configs[1..3]'s shape (4,50), configs[3]'s (4,200), configs[4]'s (7,100)
    ("n4s50", 4, 50, 1024, 100_000),
    ("n4s200", 4, 200, 256, 200_000),
    ("n7s100", 7, 100, 256, 300_000),
]


def gen_episode(name, n, s, max_steps, seed, episode, deterministic, wseed=0, td=True, n_td=10):
    """A whole Muzero._play_game episode (Muzero.py:153-207) of the reference, with every network
    call recorded per search, so the self-play driver can be replayed bit-exactly."""
    from Muzero import Muzero

    env = TowersOfHanoi(N=n, max_steps=max_steps)
    torch.manual_seed(wseed)
    np.random.seed(seed)
    mz = Muzero(env=env, s_space_size=3 * n, n_action=6, discount=0.8, dirichlet_alpha=0.25,
                n_mcts_simulations=s, unroll_n_steps=5, batch_s=256, TD_return=td, n_TD_step=n_td,
                lr=0.002, buffer_size=1000, priority_replay=True, device="cpu")
    torch.manual_seed(wseed)
    net = MuZeroNet(rpr_input_s=3 * n, action_s=6, lr=0.002, device="cpu", TD_return=td)
    rec = Recorder(net)
    mz.networks = rec
    mz.mcts = TracingMCTS(discount=0.8, root_dirichlet_alpha=0.25, n_simulations=s, batch_s=256, device="cpu")
    visits, mm = [], []
    orig = mz.mcts.run_mcts

    def run(*a, **k):
        out = orig(*a, **k)
        visits.append(mz.mcts.last_visits.astype(np.int32))
        mm.append((mz.mcts.min_max_stats.maximum, mz.mcts.min_max_stats.minimum))
        return out

    mz.mcts.run_mcts = run
    steps, states, rwds, actions, pi_probs, returns, priorities = mz._play_game(episode=episode,
                                                                                deterministic=deterministic)
    calls = rec.calls
    assert len(calls) == steps * (s + 1)
    out_pi = np.array([c[3][2] for c in calls], np.float32).reshape(steps, s + 1, 6)
    out_rwd = np.array([c[3][1] for c in calls], np.float64).reshape(steps, s + 1)
    out_v = np.array([c[3][3] for c in calls], np.float64).reshape(steps, s + 1)
    obs = np.array([c[1] for c in calls[:: s + 1]], np.float64)
    np.savez_compressed(
        os.path.join(HERE, f"episode_{name}.npz"), n=n, s=s, max_steps=max_steps, seed=seed, episode=episode,
        deterministic=int(deterministic), td=int(td), n_td=n_td, init_state_idx=env.init_state_idx,
        steps=steps, obs=obs, out_pi=out_pi, out_rwd=out_rwd, out_v=out_v, visits=np.array(visits),
        mm=np.array(mm, np.float64), states=states, rwds=rwds, actions=actions, pi_probs=pi_probs,
        returns=returns, priorities=np.asarray(priorities, np.float32),
        post_rng=np.random.random_sample(4),  # pins the RNG position after the episode
    )


def _split_calls(calls):
    """Recorder calls -> one record per run_mcts: (obs, root_pi, pi[S,6], reward[S], value[S])"""
    runs, cur = [], None
    for kind, x, a, out in calls:
        if kind == "i":
            cur = dict(obs=np.asarray(x, np.float64).reshape(-1), root_pi=np.asarray(out[2], np.float32), pi=[],
                       reward=[], value=[])
            runs.append(cur)
        else:
            cur["pi"].append(np.asarray(out[2], np.float32))
            cur["reward"].append(np.float32(out[1]))
            cur["value"].append(np.float32(out[3]))
    return runs


def _pack_runs(runs):
    """flatten per-run recorded outputs (the replay network of the tests consumes them in order)"""
    S = np.array([len(r["pi"]) for r in runs], np.int32)
    cat = lambda k, shape: (np.concatenate([np.asarray(r[k], np.float32).reshape((-1,) + shape) for r in runs])
                            if S.sum() else np.zeros((0,) + shape, np.float32))
    return dict(run_S=S, run_obs=np.array([r["obs"] for r in runs]), run_root_pi=np.array([r["root_pi"] for r in runs]),
                run_pi=cat("pi", (6,)), run_reward=cat("reward", ()), run_value=cat("value", ()))


class _ActingMCTS(TracingMCTS):
    """records every run_mcts result (action, root Q, MinMaxStats after the call)"""

    def run_mcts(self, state, network, temperature, deterministic):
        out = super().run_mcts(state, network, temperature, deterministic)
        self.trace.append((int(out[0]), float(out[2]), self.min_max_stats.maximum, self.min_max_stats.minimum))
        return out


def _traced_env(n, max_steps):
    """TowersOfHanoi whose step() results are recorded (illegal flags, rewards)"""
    env = TowersOfHanoi(N=n, max_steps=max_steps)
    env.trace = []
    orig = env.step

    def step(a):
        out = orig(a)
        env.trace.append((int(a), float(out[1]), int(out[2]), int(out[3])))
        return out

    env.step = step
    return env


def gen_acting(name, n, budgets, episodes, start, temperature, max_steps, seed, wseed=0):
    """acting_experiments/acting_ablations.py:72-128 get_results of the reference: ONE MCTS instance
    for every budget and episode (MinMaxStats carried across all of them), starts from
    get_starting_state (ES/MS/LS, :49-68) or random_reset (env/hanoi.py:98-109), every network
    output recorded per run_mcts call."""
    sys.path.insert(0, os.path.join(REF, "acting_experiments"))
    import acting_ablations as aa

    net = make_net(n, wseed)
    rec = Recorder(net)
    env = _traced_env(n, max_steps)
    label = aa.get_starting_state(env, start)
    mcts = _ActingMCTS(discount=0.8, root_dirichlet_alpha=0.25, n_simulations=budgets[0], batch_s=256, device="cpu")
    mcts.trace = []
    np.random.seed(seed)
    data = aa.get_results(env, start, rec, mcts, episodes, budgets, temperature)
    runs = _split_calls(rec.calls)
    tr = np.array(mcts.trace, np.float64).reshape(-1, 4)
    et = np.array(env.trace, np.float64).reshape(-1, 4)
    np.savez_compressed(
        os.path.join(HERE, f"acting_{name}.npz"), n=n, budgets=np.array(budgets, np.int32), episodes=episodes,
        start=-1 if start is None else start, start_label=label, temperature=temperature, max_steps=max_steps,
        seed=seed, wseed=wseed, init_state_idx=env.init_state_idx, data=np.array(data, np.float64),
        actions=tr[:, 0].astype(np.int32), root_q=tr[:, 1], mm=tr[:, 2:], env_rwd=et[:, 1],
        env_done=et[:, 2].astype(np.int32), env_illegal=et[:, 3].astype(np.int32), **_pack_runs(runs),
        post_rng=np.random.random_sample(4))


def gen_illegal(name, n, n_sims, episodes, temperature, fixed_start, max_steps, seed, wseed=0, init_state_idx=0):
    """illegal_move_rate_comparison.py:27-50 illegal_move_rate of the reference (per-episode rates,
    their mean and standard error), every network output recorded."""
    import illegal_move_rate_comparison as imr

    net = make_net(n, wseed)
    rec = Recorder(net)
    env = _traced_env(n, max_steps)
    env.init_state_idx = init_state_idx
    mcts = _ActingMCTS(discount=0.8, root_dirichlet_alpha=0.25, n_simulations=n_sims, batch_s=1, device="cpu")
    mcts.trace = []
    np.random.seed(seed)
    mean, sem = imr.illegal_move_rate(env, rec, mcts, episodes=episodes, temperature=temperature,
                                      fixed_start=fixed_start)
    runs = _split_calls(rec.calls)
    tr = np.array(mcts.trace, np.float64).reshape(-1, 4)
    et = np.array(env.trace, np.float64).reshape(-1, 4)
    np.savez_compressed(
        os.path.join(HERE, f"illegal_{name}.npz"), n=n, n_sims=n_sims, episodes=episodes, temperature=temperature,
        fixed_start=int(fixed_start), max_steps=max_steps, seed=seed, wseed=wseed, init_state_idx=init_state_idx,
        mean=mean, sem=sem, actions=tr[:, 0].astype(np.int32), mm=tr[:, 2:], env_done=et[:, 2].astype(np.int32),
        env_illegal=et[:, 3].astype(np.int32), **_pack_runs(runs), post_rng=np.random.random_sample(4))


def gen_ucb_rules(n_rows=1000, seed=41):
    """child_U (MCTS/node.py:105-123) under the two NumPy promotion rules.  The reference pins
    numpy==1.25.2 (requirements.txt:17): np.float32 prior * Python-float w is promoted to float64 and
    rounded once into the float32 array, fl32(fl64(prior) * w); NumPy >= 2 (NEP 50, this container)
    keeps float32: fl32(prior * fl32(w)).  Rows are (N_parent, N_child, prior) triples drawn at random;
    the reference's own child_U (run here, NumPy 2) pins the NumPy-2 column, the NumPy-1 column is the
    stated rule evaluated explicitly (no NumPy-1 run is possible here: parity unpinned for it)."""
    import math

    from MCTS.node import Node

    class Cfg:
        pb_c_base, pb_c_init = 19652, 1.25

    rs = np.random.RandomState(seed)
    rows = []
    for _ in range(n_rows):
        npar = int(rs.randint(1, 400))
        prior = rs.dirichlet(np.ones(6)).astype(np.float32)
        parent = Node(prior=None)
        parent.expand(prior, None, 0.0)
        parent.N = npar
        nc = rs.randint(0, npar, 6)
        for c, k in zip(parent.children, nc):
            c.N = int(k)
        u_ref = parent.child_U(Cfg)  # the reference, NumPy 2 semantics
        for c, k, u2 in zip(parent.children, nc, u_ref):
            w = (math.log((npar + 19652 + 1) / 19652) + 1.25) * math.sqrt(npar) / (int(k) + 1)
            np2 = np.float32(np.float32(c.prior) * np.float32(w))
            np1 = np.float32(np.float64(c.prior) * w)
            assert np2 == u2
            rows.append((npar, int(k), float(c.prior), float(np1), float(np2)))
    a = np.array(rows, np.float64)
    differ = a[:, 3] != a[:, 4]
    np.savez_compressed(os.path.join(HERE, "ucb_np1_vs_np2.npz"), n_parent=a[:, 0].astype(np.int32),
                        n_child=a[:, 1].astype(np.int32), prior=a[:, 2].astype(np.float32),
                        u_np1=a[:, 3].astype(np.float32), u_np2=a[:, 4].astype(np.float32), differ=differ)
    return int(differ.sum()), len(rows)


def gen_tie_replay(n=3, s=12, n_roots=4, seed=51, wseed=0):
    """A run_mcts trace that meets argmax ties beyond the root's first selection: the recorded
    network returns uniform priors, so every freshly expanded node's first selection is a 6-way
    tie (MCTS/node.py:83-86).  np.random.choice over an argmax set is replaced (in this script)
    by the LOWEST index -- the resolution the kernels apply to such extra ties -- so the trace is
    the reference's tree under that resolution; the number of multi-candidate argmax choices per
    root is recorded (the kernels count all but the root's first as extra_ties)."""
    net = make_net(n, wseed)

    class UniformRecorder(Recorder):
        def initial_inference(self, x):
            h, r, pi, v = self.net.initial_inference(x)
            out = (h, r, np.full(6, 1.0 / 6.0, np.float32), v)
            self.calls.append(("i", x.numpy().copy(), -1, out))
            return out

        def recurrent_inference(self, h, a):
            h2, r, pi, v = self.net.recurrent_inference(h, a)
            out = (h2, r, np.full(6, 1.0 / 6.0, np.float32), v)
            self.calls.append(("r", h.numpy().copy(), int(a.argmax()), out))
            return out

    orig = np.random.choice
    ties = []

    def lowest(a, *args, **kw):
        if "p" in kw or isinstance(a, (int, np.integer)):
            return orig(a, *args, **kw)
        ties[-1] += int(len(a) > 1)
        return int(np.min(a))

    env = TowersOfHanoi(N=n, max_steps=200)
    rs = np.random.RandomState(seed)
    roots = [int(i) for i in rs.randint(0, 3 ** n - 1, n_roots)]
    out = dict(visits=[], rootQ=[], mm=[], pi=[], root_pi=[], rwd=[], value=[], obs=[])
    np.random.seed(seed)
    np.random.choice = lowest
    try:
        for idx in roots:
            ties.append(0)
            mcts = TracingMCTS(discount=0.8, root_dirichlet_alpha=0.0, n_simulations=s, batch_s=1, device="cpu")
            obs = np.zeros(3 * n)
            obs[np.arange(n) * 3 + np.array(env.states[idx])] = 1.0
            rec = UniformRecorder(net)
            _, pi, q = mcts.run_mcts(obs, rec, 1.0, True)
            run = _split_calls(rec.calls)[0]
            out["visits"].append(mcts.last_visits.astype(np.int32))
            out["rootQ"].append(float(q))
            out["mm"].append((mcts.min_max_stats.maximum, mcts.min_max_stats.minimum))
            out["pi"].append(np.array(run["pi"], np.float32))
            out["root_pi"].append(run["root_pi"])
            out["rwd"].append(np.array(run["reward"], np.float32))
            out["value"].append(np.array(run["value"], np.float32))
            out["obs"].append(obs)
    finally:
        np.random.choice = orig
    np.savez_compressed(os.path.join(HERE, "tie_replay.npz"), n=n, s=s, root_idx=np.array(roots, np.int32),
                        obs=np.array(out["obs"]), visits=np.array(out["visits"]), rootQ=np.array(out["rootQ"]),
                        mm=np.array(out["mm"]), root_pi=np.array(out["root_pi"]), pi=np.array(out["pi"]),
                        rwd=np.array(out["rwd"]), value=np.array(out["value"]), ties=np.array(ties, np.int32))
    return ties


def gen_random_reset(seed=61):
    """TowersOfHanoi.random_reset (env/hanoi.py:98-109): the start states a seeded global stream
    gives, for N = 3 and N = 4 and goal pegs 2 / 0, and the stream position after them."""
    np.random.seed(seed)
    recs = []
    for n, goal in ((3, 2), (4, 2), (3, 0)):
        env = TowersOfHanoi(N=n, max_steps=10, goal_peg=goal)
        for _ in range(40):
            env.random_reset()
            recs.append((n, goal, state_index(env.c_state, n)))
    a = np.array(recs, np.int32)
    np.savez_compressed(os.path.join(HERE, "random_reset.npz"), seed=seed, n=a[:, 0], goal_peg=a[:, 1],
                        state_idx=a[:, 2], post_rng=np.random.random_sample(4))


ACTING_CASES = [
    # name, n, budgets, episodes, start, temperature, max_steps, seed
    ("es_t1", 3, [1, 3, 5], 2, 0, 1.0, 30, 21),
    ("rand_t05", 3, [2, 4], 3, None, 0.5, 25, 22),
]
ILLEGAL_CASES = [
    # name, n, n_sims, episodes, temperature, fixed_start, max_steps, seed
    ("rand_t0", 3, 5, 4, 0.0, False, 25, 31),
    ("fixed_t1", 3, 3, 3, 1.0, True, 20, 32),
]


def gen_checkpoint():
    """A muzero_model.pt in the reference's format (training_main.py:91-103) after one Adam step,
    plus the weights after the reference's own head ablation (acting_ablations.py:29-45)."""
    sys.path.insert(0, os.path.join(REF, "acting_experiments"))
    net = make_net(3, 2)
    x = torch.zeros(4, 9)
    x[:, 0] = 1
    loss = net.represent(x).sum() + sum(p.sum() for p in net.prediction(net.represent(x)))
    net.update(loss)
    torch.save({"Muzero_net": net.state_dict(), "Net_optim": net.optimiser.state_dict()},
               os.path.join(HERE, "muzero_model_N3.pt"))
    torch.manual_seed(123)
    net.policy_net.apply(net.reset_param)
    net.rwd_net.apply(net.reset_param)
    np.savez_compressed(os.path.join(HERE, "ablated_N3.npz"),
                        **{k: v.numpy() for k, v in net.state_dict().items() if k.startswith(("policy", "rwd"))})


def gen_training(name, n, td, priority, updates=3, buffer_size=96, batch_s=24, seed=11, wseed=5, full=True):
    """Muzero._update (Muzero.py:209-274) + Buffer (buffer.py) of the reference: a buffer filled
    with seeded synthetic transitions, then `updates` rounds of {sample, _update,
    update_priorities}; records the sampled indices / IS weights, the three losses, the new
    priorities and every parameter after each update (and the Adam state at the end)."""
    from Muzero import Muzero

    env = TowersOfHanoi(N=n, max_steps=200)
    torch.manual_seed(wseed)
    mz = Muzero(env=env, s_space_size=3 * n, n_action=6, discount=0.8, dirichlet_alpha=0.25,
                n_mcts_simulations=5, unroll_n_steps=5, batch_s=batch_s, TD_return=td, n_TD_step=10,
                lr=0.002, buffer_size=buffer_size, priority_replay=priority, device="cpu")
    # initial weights: torch.manual_seed(wseed) then the MuZeroNet constructor (the test rebuilds them)
    g = np.random.default_rng(seed)
    T = 70  # > buffer_size: exercises the ring wrap-around of Buffer._add
    st = g.integers(0, 3, (T, n))
    states = np.zeros((T, 3 * n), np.float32)
    states[np.arange(T)[:, None], np.arange(n) * 3 + st] = 1
    rwds = np.where(g.random((T, 5)) < 0.1, 100.0, np.where(g.random((T, 5)) < 0.3, -0.1, 0.0)).astype(np.float32)
    actions = g.integers(0, 6, (T, 5)).astype(np.int64)
    pi_probs = g.dirichlet(np.ones(6), size=(T, 5)).astype(np.float32)
    returns = g.normal(0.0, 20.0, (T, 5)).astype(np.float32)
    prios = (g.random(T) + 0.05).astype(np.float32)
    for a, b in ((0, 40), (40, 70), (0, 50)):  # three adds, the last wraps the ring
        mz.buffer.add(states[a:b], rwds[a:b], actions[a:b], pi_probs[a:b], returns[a:b], prios[a:b])
    buf0 = dict(b_states=mz.buffer.states.copy(), b_rwds=mz.buffer.rwds.copy(), b_actions=mz.buffer.actions.copy(),
                b_pi=mz.buffer.pi_probs.copy(), b_returns=mz.buffer.mc_returns.copy(),
                b_prios=mz.buffer.priorities.copy(), b_ptr=mz.buffer.ptr, b_full=int(mz.buffer.is_full))
    np.random.seed(seed)
    rec = {k: [] for k in ("indx", "isw", "v_loss", "r_loss", "p_loss", "new_prio")}
    params = []
    for _ in range(updates):
        if priority:
            bs, br, ba, bp, bret, indx, w = mz.buffer.priority_sample(batch_s)
        else:
            bs, br, ba, bp, bret = mz.buffer.uniform_sample(batch_s)
            indx, w = None, None
        newp, vl, rl, pl = mz._update(bs, br, ba, bp, bret, w)
        mz.buffer.update_priorities(indx, newp)
        rec["indx"].append(np.full(batch_s, -1) if indx is None else indx)
        rec["isw"].append(np.zeros(batch_s, np.float32) if w is None else w.numpy())
        rec["new_prio"].append(np.zeros(batch_s, np.float32) if newp is None else newp)
        rec["v_loss"].append(float(vl))
        rec["r_loss"].append(float(rl))
        rec["p_loss"].append(float(pl))
        params.append(np.concatenate([v.detach().numpy().reshape(-1) for v in mz.networks.state_dict().values()]))
    opt_state = mz.networks.optimiser.state_dict()["state"]
    exp_avg = np.concatenate([opt_state[i]["exp_avg"].numpy().reshape(-1) for i in sorted(opt_state)])
    exp_avg_sq = np.concatenate([opt_state[i]["exp_avg_sq"].numpy().reshape(-1) for i in sorted(opt_state)])
    params = np.array(params, np.float64)
    extra = dict(final_params=params[-1].astype(np.float32), exp_avg=exp_avg, exp_avg_sq=exp_avg_sq) if full else {}
    np.savez_compressed(
        os.path.join(HERE, f"training_{name}.npz"), n=n, td=int(td), priority=int(priority), seed=seed, wseed=wseed,
        batch_s=batch_s, buffer_size=buffer_size, updates=updates, **buf0,
        **{k: np.array(v) for k, v in rec.items()},
        param_sum=params.sum(1), param_sumsq=(params ** 2).sum(1), **extra,
        final_prios=mz.buffer.priorities.copy(), post_rng=np.random.random_sample(4))


TRAINING_CASES = [("n3_td_prio", 3, True, True, True), ("n4_mc_uniform", 4, False, False, False)]


EPISODE_CASES = [
    ("n3s25_t1", 3, 25, 40, 3, 1, False),
    ("n3s25_t05", 3, 25, 30, 5, 600, False),
    ("n3s10_det", 3, 10, 25, 7, 900, True),
]


def main():
    if "--policy-only" in sys.argv:
        gen_play_policy()
        gen_bad_temperature()
        for name, n, s_, roots, det, alpha, t, extra in REPLAY_CASES:
            if "_t0" in name[-4:] or name.endswith(("_t03", "_t07", "_t09")):
                gen_replay(name, n, s_, roots, det, alpha, t, **extra)
        return
    if "--agree-only" in sys.argv:
        for c in AGREE_CASES:
            gen_agreement(*c)
        print(gen_agreement_trace(*AGREE_CASES[1]))
        return
    if "--agree-trace" in sys.argv:
        print(gen_agreement_trace(*AGREE_CASES[1]))
        return
    if "--corners-only" in sys.argv:
        print("ucb rows differing", gen_ucb_rules())
        print("tie counts", gen_tie_replay())
        gen_random_reset()
        return
    if "--acting-only" in sys.argv:
        for c in ACTING_CASES:
            gen_acting(*c)
        for c in ILLEGAL_CASES:
            gen_illegal(*c)
        return
    gen_ucb_rules()
    gen_tie_replay()
    gen_random_reset()
    gen_play_policy()
    gen_bad_temperature()
    for c in AGREE_CASES:
        gen_agreement(*c)
    gen_agreement_trace(*AGREE_CASES[1])
    for c in ACTING_CASES:
        gen_acting(*c)
    for c in ILLEGAL_CASES:
        gen_illegal(*c)
    for name, n, td, prio, full in TRAINING_CASES:
        gen_training(name, n, td, prio, full=full)
    gen_checkpoint()
    for name, n, s, ms, seed, ep, det in EPISODE_CASES:
        gen_episode(name, n, s, ms, seed, ep, det)
    for n in (3, 4, 7):
        gen_env(n)
        gen_solver(n)
    gen_env_maxsteps()
    for n in (3, 4, 7):
        gen_mlp(n, 0)
    gen_mlp(3, 0, td=False)
    gen_mlp(4, 1)
    summary = {}
    for name, n, s, roots, det, alpha, t, extra in REPLAY_CASES:
        ch = gen_replay(name, n, s, roots, det, alpha, t, **extra)
        ties = ch[(ch[:, 2] == 0) & (ch[:, 1] > 1)]
        summary[name] = {"choice_calls": int(len(ch)), "multi_candidate_ties": int(len(ties)),
                         "tie_sizes": sorted(set(int(v) for v in ties[:, 1]))}
    with open(os.path.join(HERE, "rng_order.json"), "w") as f:
        json.dump({
            "order_per_run_mcts": [
                "np.random.dirichlet(np.ones(6,float32)*alpha) if not deterministic and alpha>0 and eps>0 (MCTS/mcts.py:57-66,149)",
                "np.random.choice(argmax-set) at EVERY best_child (MCTS/node.py:86); a 1-element set draws nothing",
                "np.random.choice(6, p=pi) -> one random_sample() double if not deterministic (MCTS/mcts.py:118-120)",
            ],
            "observed": summary,
            "numpy": np.__version__, "torch": torch.__version__,
        }, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
