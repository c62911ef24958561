"""Training update: Buffer (buffer.py) + Muzero._update (Muzero.py:209-274)
against fixtures recorded from the reference itself (tests/golden/gen_golden.py gen_training):
same initial weights (torch.manual_seed), same synthetic transitions, same NumPy RNG seed ->
same sampled indices / importance weights (exact), losses, new priorities, parameters and Adam
moments.  On the CPU the update is the reference's torch op sequence: in the build container that
recorded the fixtures it reproduces them bit for bit, on another host CPU torch's vectorised
reductions may differ in the last ulp, so float results are checked at fp32-rounding tolerance;
on the GPU (PyTorch-ROCm GEMMs, other reduction orders) at fp32 tolerances."""
import numpy as np
import pytest
import torch

from conftest import golden

CASES = ["n3_td_prio", "n4_mc_uniform"]


def synthetic_transitions(n, seed, T=70):
    """the generator's inputs (gen_training), re-made from its seed"""
    g = np.random.default_rng(seed)
    st = g.integers(0, 3, (T, n))
    states = np.zeros((T, 3 * n), np.float32)
    states[np.arange(T)[:, None], np.arange(n) * 3 + st] = 1
    rwds = np.where(g.random((T, 5)) < 0.1, 100.0, np.where(g.random((T, 5)) < 0.3, -0.1, 0.0)).astype(np.float32)
    actions = g.integers(0, 6, (T, 5)).astype(np.int64)
    pi_probs = g.dirichlet(np.ones(6), size=(T, 5)).astype(np.float32)
    returns = g.normal(0.0, 20.0, (T, 5)).astype(np.float32)
    prios = (g.random(T) + 0.05).astype(np.float32)
    return states, rwds, actions, pi_probs, returns, prios


def _host(x):
    return x.cpu().numpy() if torch.is_tensor(x) else x


def run_case(g, device, impl="torch"):
    from muzero_hanoi_amd.muzero import Muzero

    n, td, prio = int(g["n"]), bool(g["td"]), bool(g["priority"])
    torch.manual_seed(int(g["wseed"]))
    mz = Muzero(env=None, s_space_size=3 * n, n_action=6, discount=0.8,
                dirichlet_alpha=0.25, n_mcts_simulations=5, unroll_n_steps=5, batch_s=int(g["batch_s"]), TD_return=td,
                n_TD_step=10, lr=0.002, buffer_size=int(g["buffer_size"]), priority_replay=prio, device=device,
                update_impl=impl)
    data = synthetic_transitions(n, int(g["seed"]))
    for a, b in ((0, 40), (40, 70), (0, 50)):
        mz.buffer.add(*(x[a:b] for x in data))
    buf = mz.buffer
    assert (buf.ptr, int(buf.is_full)) == (int(g["b_ptr"]), int(g["b_full"]))
    for name, arr in (("b_states", buf.states), ("b_rwds", buf.rwds), ("b_actions", buf.actions), ("b_pi", buf.pi_probs),
                      ("b_returns", buf.mc_returns)):
        assert np.array_equal(arr.cpu().numpy(), g[name]), name
    assert np.array_equal(buf.priorities, g["b_prios"])
    np.random.seed(int(g["seed"]))
    out = {k: [] for k in ("indx", "isw", "v_loss", "r_loss", "p_loss", "new_prio", "param_sum", "param_sumsq")}
    for _ in range(int(g["updates"])):
        if prio:
            s, r, a, p, ret, indx, w = buf.priority_sample(int(g["batch_s"]))
        else:
            s, r, a, p, ret = buf.uniform_sample(int(g["batch_s"]))
            indx, w = None, None
        newp, vl, rl, pl = mz._update(s, r, a, p, ret, w)
        buf.update_priorities(indx, newp)
        # with the fused update the buffer draws on the device: indices / new priorities as device tensors
        out["indx"].append(np.full(int(g["batch_s"]), -1) if indx is None else _host(indx))
        out["isw"].append(np.zeros(int(g["batch_s"]), np.float32) if w is None else w.cpu().numpy())
        out["new_prio"].append(np.zeros(int(g["batch_s"]), np.float32) if newp is None else _host(newp))
        for k, v in (("v_loss", vl), ("r_loss", rl), ("p_loss", pl)):
            out[k].append(float(v))
        flat = torch.cat([v.detach().reshape(-1) for v in mz.networks.state_dict().values()]).double().cpu().numpy()
        out["param_sum"].append(flat.sum())
        out["param_sumsq"].append((flat ** 2).sum())
    st = mz.networks.optimiser.state_dict()["state"]
    out["final_params"] = flat.astype(np.float32)
    out["exp_avg"] = torch.cat([st[i]["exp_avg"].reshape(-1) for i in sorted(st)]).cpu().numpy()
    out["exp_avg_sq"] = torch.cat([st[i]["exp_avg_sq"].reshape(-1) for i in sorted(st)]).cpu().numpy()
    out["final_prios"] = buf.priorities.copy()
    out["post_rng"] = np.random.random_sample(4)
    return out


@pytest.mark.parametrize("case", CASES)
def test_buffer_and_update_vs_reference_on_cpu(case):
    g = golden(f"training_{case}.npz")
    torch.set_num_threads(1)
    out = run_case(g, "cpu")
    for k in ("indx", "isw", "post_rng"):  # the RNG stream and the sampling math: exact
        assert np.array_equal(np.array(out[k]), g[k]), k
    for k in ("v_loss", "r_loss", "p_loss"):
        np.testing.assert_allclose(np.array(out[k]), g[k], rtol=1e-5, err_msg=k)
    np.testing.assert_allclose(np.array(out["new_prio"]), g["new_prio"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(out["final_prios"], g["final_prios"], rtol=1e-4, atol=1e-4)
    # a gradient at rounding noise can flip Adam's first steps (each moves ~lr * sign(g)):
    # the parameter sum then moves by ~2 lr per flipped parameter
    np.testing.assert_allclose(np.array(out["param_sum"]), g["param_sum"], rtol=1e-6, atol=8 * 0.002)
    if "final_params" in g.files:
        d = np.abs(out["final_params"] - g["final_params"])
        assert (d < 1e-5).mean() > 0.99 and d.max() < 6 * 0.002, (float((d < 1e-5).mean()), float(d.max()))
        m = np.abs(out["exp_avg"] - g["exp_avg"]) <= 1e-3 * np.abs(g["exp_avg"]) + 1e-5
        assert m.mean() > 0.9, float(m.mean())


@pytest.mark.gpu
@pytest.mark.parametrize("impl", ["torch", "graph", "fused"])
@pytest.mark.parametrize("case", CASES)
def test_update_on_gpu_vs_reference(case, impl):
    """PyTorch-ROCm update vs the reference's CPU update: same samples, losses and priorities to
    fp32 reduction-order tolerance; parameters after 3 Adam steps within a few lr of each other
    only where a gradient sits at the rounding noise (Adam's first steps move by ~lr * sign(g))."""
    g = golden(f"training_{case}.npz")
    out = run_case(g, "cuda", impl=impl)
    for k in ("indx", "post_rng"):
        assert np.array_equal(np.array(out[k]), g[k]), k
    np.testing.assert_allclose(np.array(out["isw"]), g["isw"], rtol=1e-6)
    for k in ("v_loss", "r_loss", "p_loss"):
        np.testing.assert_allclose(np.array(out[k]), g[k], rtol=2e-4, err_msg=k)
    np.testing.assert_allclose(np.array(out["new_prio"]), g["new_prio"], rtol=1e-3, atol=1e-3)
    np.testing.assert_allclose(np.array(out["param_sum"]), g["param_sum"], rtol=1e-5, atol=8 * 0.002)
    if "final_params" in g.files:
        d = np.abs(out["final_params"] - g["final_params"])
        assert (d < 1e-5).mean() > 0.99 and d.max() < 6 * 0.002, (float((d < 1e-5).mean()), float(d.max()))


@pytest.mark.gpu
@pytest.mark.parametrize("impl", ["torch", "fused"])
def test_training_loop_runs_on_gpu(impl):
    """Muzero.training_loop (Muzero.py:81-151) end to end: self-play searches on the fused kernel,
    buffer on the device, updates on PyTorch-ROCm (or the fused HIP update with the draw and the
    priority write-back on the device), and the search sees the updated weights."""
    from muzero_hanoi_amd.env import TowersOfHanoi
    from muzero_hanoi_amd.muzero import Muzero

    torch.manual_seed(0)
    np.random.seed(0)
    mz = Muzero(env=TowersOfHanoi(N=3, max_steps=300), s_space_size=9, n_action=6, discount=0.8, dirichlet_alpha=0.25,
                n_mcts_simulations=8, unroll_n_steps=5, batch_s=16, TD_return=True, n_TD_step=10, lr=0.002,
                buffer_size=400, priority_replay=True, device="cuda", update_impl=impl)
    assert mz.buffer.device_sampling == (impl == "fused")
    before = {k: v.detach().clone() for k, v in mz.networks.state_dict().items()}
    acc = mz.training_loop(n_loops=17, min_replay_size=0, print_acc=8)
    assert len(acc) == 2 and all(np.isfinite(acc))
    assert len(mz.buffer) > 0  # some episodes reached the goal
    moved = any(not torch.equal(before[k], v) for k, v in mz.networks.state_dict().items())
    assert moved
    action, pi, q = mz.mcts.run_mcts(mz.env.reset(), mz.networks, temperature=1.0, deterministic=True)
    assert 0 <= action < 6 and abs(pi.sum() - 1) < 1e-9 and np.isfinite(q)


@pytest.mark.parametrize("seed", range(8))
def test_sampling_fast_path_equals_numpy_choice(seed):
    """Buffer's draw == np.random.choice(arange(n), size, replace=True[, p]) (buffer.py:79-112):
    same indices and the same global-stream position afterwards, with and without priorities."""
    from muzero_hanoi_amd.buffer import Buffer

    g = np.random.default_rng(seed)
    n = int(g.integers(1, 5000))
    buf = Buffer(n, 5, d_state=9, n_action=6, device="cpu")
    buf.priorities[:] = (g.random(n) + 0.01).astype(np.float32)
    buf.ptr, buf.is_full = 0, True
    probs = buf.priorities / np.sum(buf.priorities)
    np.random.seed(seed)
    want = np.random.choice(np.arange(n), size=64, replace=True, p=probs)
    after = np.random.random_sample()
    np.random.seed(seed)
    got = buf.priority_sample(64)[5]
    assert np.array_equal(got, want) and np.random.random_sample() == after
    np.random.seed(seed)
    want = np.random.choice(np.arange(n), size=64, replace=True)
    after = np.random.random_sample()
    np.random.seed(seed)
    st = buf.uniform_sample(64)[0]
    assert np.random.random_sample() == after and st.shape == (64, 9)
    np.random.seed(seed)
    assert np.array_equal(np.random.randint(0, n, size=64), want)


@pytest.mark.gpu
def test_fused_update_after_checkpoint_reload():
    """FusedUpdate re-transposes weights written outside it and re-binds the optimiser's state
    tensors after `load_state_dict` (training_main.py:93-103 checkpoint format): an update right
    after a reload matches the torch update from the same checkpoint."""
    import copy

    from muzero_hanoi_amd.muzero import Muzero

    def make(impl):
        torch.manual_seed(0)
        return Muzero(env=None, s_space_size=9, n_action=6, discount=0.8, dirichlet_alpha=0.25, n_mcts_simulations=5,
                      unroll_n_steps=5, batch_s=32, TD_return=True, n_TD_step=10, lr=0.002, buffer_size=200,
                      priority_replay=True, device="cuda", update_impl=impl)

    data = synthetic_transitions(3, 7, T=120)
    fused, ref = make("fused"), make("torch")
    for mz in (fused, ref):
        mz.buffer.add(*data)
    # a checkpoint taken after two torch updates
    np.random.seed(5)
    for _ in range(2):
        s, r, a, p, ret, indx, w = ref.buffer.priority_sample(32)
        ref._update(s, r, a, p, ret, w)
    ckpt = {"Muzero_net": copy.deepcopy(ref.networks.state_dict()),
            "Net_optim": copy.deepcopy(ref.networks.optimiser.state_dict())}
    # the fused agent trains on its own first, then loads the checkpoint
    np.random.seed(6)
    for _ in range(2):
        s, r, a, p, ret, indx, w = fused.buffer.priority_sample(32)
        fused._update(s, r, a, p, ret, w)
    fused.networks.load_state_dict(ckpt["Muzero_net"])
    fused.networks.optimiser.load_state_dict(ckpt["Net_optim"])
    np.random.seed(9)
    batch = fused.buffer.priority_sample(32)
    out_f = fused._update(*batch[:5], batch[6])
    out_r = ref._update(*batch[:5], batch[6])
    for x, y in zip(out_f[1:], out_r[1:]):
        np.testing.assert_allclose(float(x), float(y), rtol=2e-4)
    np.testing.assert_allclose(_host(out_f[0]), out_r[0], rtol=1e-3, atol=1e-3)
    pf = torch.cat([v.reshape(-1) for v in fused.networks.state_dict().values()]).cpu().numpy()
    pr = torch.cat([v.reshape(-1) for v in ref.networks.state_dict().values()]).cpu().numpy()
    d = np.abs(pf - pr)
    assert (d < 1e-5).mean() > 0.99 and d.max() < 6 * 0.002, (float((d < 1e-5).mean()), float(d.max()))
    sf = fused.networks.optimiser.state_dict()["state"]
    sr = ref.networks.optimiser.state_dict()["state"]
    assert all(float(sf[i]["step"]) == float(sr[i]["step"]) == 3.0 for i in sr)
