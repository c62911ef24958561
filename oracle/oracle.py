"""ctypes wrapper around oracle/_build/libmzh_oracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and only
as the checker. The product path (muzero-hanoi_amd/) never imports it.

The C restatement (mzh_oracle.c) follows env/hanoi.py:47-151, env/hanoi_utils.py:4-26,
networks.py:71-196, MCTS/mcts.py:34-176, MCTS/node.py:30-136 and MCTS/utils_mcts.py:1-16 of the
reference; it is pinned against the fixtures in tests/golden/ (generated from the reference).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libmzh_oracle.so")

WEIGHT_KEYS = [
    f"{net}.{layer}.{kind}"
    for net in ("representation_net", "dynamic_net", "rwd_net", "policy_net", "value_net")
    for layer in (0, 2)
    for kind in ("weight", "bias")
]

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
        L = _lib
        L.orc_expf.restype = ctypes.c_float
        L.orc_expf.argtypes = [ctypes.c_float]
        L.orc_signed_parabolic.restype = ctypes.c_float
        L.orc_signed_parabolic.argtypes = [ctypes.c_float]
        L.orc_logits_to_value.restype = ctypes.c_float
        L.orc_logits_to_value.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_logits_expectation.restype = ctypes.c_float
        L.orc_logits_expectation.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_markstein_mismatches.restype = ctypes.c_long
        L.orc_markstein_mismatches.argtypes = [ctypes.c_long, ctypes.c_uint64]
        L.orc_ucb_table.restype = ctypes.c_double
        L.orc_ucb_table.argtypes = [ctypes.c_int]
        L.orc_hanoi_solver.restype = ctypes.c_long
        L.orc_hanoi_solver.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        L.orc_legal_mask.restype = ctypes.c_int
        L.orc_legal_mask.argtypes = [ctypes.c_int, ctypes.c_void_p]
        L.orc_env_step.restype = ctypes.c_int
        L.orc_env_step.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                   ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_weights_size.restype = ctypes.c_size_t
        L.orc_weights_size.argtypes = [ctypes.c_int, ctypes.c_int]
        L.orc_initial_inference.restype = None
        L.orc_initial_inference.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 7
        L.orc_recurrent_inference.restype = None
        L.orc_recurrent_inference.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 9
        L.orc_play_policy.restype = ctypes.c_int
        L.orc_play_policy.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_int, ctypes.c_double, ctypes.c_void_p,
                                      ctypes.c_void_p]
        L.orc_search.restype = ctypes.c_int
        L.orc_search.argtypes = (
            [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_void_p,
             ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p,
             ctypes.c_double, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_void_p] * 10)
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _c(a, dt):
    return None if a is None else np.ascontiguousarray(a, dtype=dt)


def flat_weights(weights):
    """dict(state_dict key -> array) -> canonical flat fp32 vector (include/mzh.h)."""
    return np.concatenate([np.asarray(weights[k], np.float32).reshape(-1) for k in WEIGHT_KEYS])


def load_weights_npz(path):
    z = np.load(path)
    w = {k: z[k] for k in WEIGHT_KEYS}
    support = w["value_net.2.bias"].shape[0]
    in_dim = w["representation_net.0.weight"].shape[1]
    return w, in_dim, support


def expf(x):
    return lib().orc_expf(float(x))


def logits_to_value(logits):
    """logits_to_transformed_expected_value of one logit row (networks.py:152-189)"""
    lg = _c(logits, np.float32)
    return float(lib().orc_logits_to_value(_p(lg), lg.size))


def logits_expectation(logits):
    """the pre-transform expected scalar of one logit row (networks.py:174-184)"""
    lg = _c(logits, np.float32)
    return float(lib().orc_logits_expectation(_p(lg), lg.size))


def signed_parabolic(x):
    """_signed_parabolic (networks.py:186-189) with a correctly rounded sqrt, fp32 op by op"""
    return float(lib().orc_signed_parabolic(float(x)))


def ucb_table(n):
    return np.array([lib().orc_ucb_table(i) for i in range(n)], np.float64)


def hanoi_solver(state, goal_peg=2):
    st = np.ascontiguousarray(state, np.uint8)
    return int(lib().orc_hanoi_solver(len(st), _p(st), goal_peg))


def legal_mask(state):
    st = np.ascontiguousarray(state, np.uint8)
    return int(lib().orc_legal_mask(len(st), _p(st)))


def env_step(state, action, ctr, active, max_steps, goal_peg=2):
    """One TowersOfHanoi.step. Returns (code, new_state, moved, ctr, active, done, illegal)."""
    st = np.array(state, np.uint8)
    moved = np.zeros_like(st)
    c = ctypes.c_int(ctr)
    act = ctypes.c_uint8(active)
    done = ctypes.c_uint8(0)
    ill = ctypes.c_uint8(0)
    code = lib().orc_env_step(len(st), goal_peg, max_steps, _p(st), int(action), _p(moved),
                              ctypes.byref(c), ctypes.byref(act), ctypes.byref(done), ctypes.byref(ill))
    return code, st, moved, c.value, act.value, done.value, ill.value


def initial_inference(flat, in_dim, support, x):
    x = _c(x, np.float32)
    B = x.shape[0]
    h = np.zeros((B, 64), np.float32)
    r = np.zeros(B, np.float32)
    pi = np.zeros((B, 6), np.float32)
    v = np.zeros(B, np.float32)
    pl = np.zeros((B, 6), np.float32)
    vl = np.zeros((B, support), np.float32)
    flat = _c(flat, np.float32)
    lib().orc_initial_inference(_p(flat), in_dim, support, B, _p(x), _p(h), _p(r), _p(pi), _p(v), _p(pl), _p(vl))
    return dict(h=h, reward=r, pi=pi, value=v, policy_logits=pl, value_logits=vl)


def recurrent_inference(flat, in_dim, support, h_in, actions):
    h_in = _c(h_in, np.float32)
    a = _c(actions, np.int32)
    B = h_in.shape[0]
    h = np.zeros((B, 64), np.float32)
    r = np.zeros(B, np.float32)
    pi = np.zeros((B, 6), np.float32)
    v = np.zeros(B, np.float32)
    pl = np.zeros((B, 6), np.float32)
    vl = np.zeros((B, support), np.float32)
    rl = np.zeros((B, support), np.float32)
    flat = _c(flat, np.float32)
    lib().orc_recurrent_inference(_p(flat), in_dim, support, B, _p(h_in), _p(a), _p(h), _p(r), _p(pi),
                                  _p(v), _p(pl), _p(vl), _p(rl))
    return dict(h=h, reward=r, pi=pi, value=v, policy_logits=pl, value_logits=vl, reward_logits=rl)


def numpy_pow_table(n_max, temperature):
    """np.power(n, exp) for n = 0..n_max exactly as generate_play_policy computes it (MCTS/mcts.py:168-174:
    an int64 array raised to a Python float), or None where no power is taken or the exponent is an
    integer (exact products).  NumPy's float64 power is vectorised (SVML on AVX-512 hosts) and differs
    from libm's pow in the last bit for some n, so the C restatement takes the values from NumPy."""
    if not 0.0 < temperature <= 1.0:
        return None
    e = max(1.0, min(5.0, 1.0 / temperature))
    if e == int(e):
        return None
    return np.power(np.arange(n_max + 1, dtype=np.int64), e)


def play_policy(visits, temperature, deterministic, u=0.0):
    v = np.ascontiguousarray(visits, np.int32)
    pi = np.zeros(6, np.float64)
    pt = _c(numpy_pow_table(int(v.max()) if v.size else 0, temperature), np.float64)
    a = lib().orc_play_policy(_p(v), float(temperature), int(deterministic), float(u), _p(pt), _p(pi))
    return a, pi


def search(n_disks, S, obs, *, flat=None, support=33, replay=None, noise=None, eps=0.25,
           tie_idx=None, action_u=None, temperature=1.0, deterministic=False, minmax_in=None,
           discount=0.8, np1_ucb=False, depths=False):
    """Batched search over B independent roots (each a fresh or given MinMaxStats).

    replay: dict(root_pi[B,6], pi[B,S,6], rwd[B,S], value[B,S]) -> tree-only mode.
    depths=True adds `depths` [B,S]: each simulation's selection depth."""
    obs = _c(obs, np.float32)
    B = obs.shape[0]
    visits = np.zeros((B, 6), np.int32)
    rootQ = np.zeros(B, np.float64)
    mm = np.zeros((B, 2), np.float64)
    et = np.zeros(B, np.int32)
    action = np.zeros(B, np.int32)
    pi = np.zeros((B, 6), np.float64)
    latent = np.full((B, S + 1), -1, np.int32)
    latent_len = np.zeros(B, np.int32)
    steps = np.zeros(B, np.int64)
    dep = np.zeros((B, S), np.int32) if depths else None
    rp = [None] * 4
    if replay is not None:
        rp = [_c(replay["root_pi"], np.float32), _c(replay["pi"], np.float32),
              _c(replay["rwd"], np.float32), _c(replay["value"], np.float32)]
    flat = _c(flat, np.float32)
    noise = _c(noise, np.float64)
    tie = _c(tie_idx if tie_idx is not None else np.zeros(B), np.int32)
    au = _c(action_u, np.float64)
    mmi = _c(minmax_in, np.float64)
    pt = _c(numpy_pow_table(S, temperature), np.float64)
    st = lib().orc_search(n_disks, S, B, float(discount), 1 if np1_ucb else 0, _p(flat), support,
                          _p(obs), _p(rp[0]), _p(rp[1]), _p(rp[2]), _p(rp[3]), _p(noise), float(eps),
                          _p(tie), _p(au), float(temperature), int(deterministic), _p(pt), _p(mmi),
                          _p(visits), _p(rootQ), _p(mm), _p(et), _p(action), _p(pi), _p(latent),
                          _p(latent_len), _p(steps), _p(dep))
    if st == -2:
        raise ValueError(f"Expect `temperature` to be in the range [0.0, 1.0], got {temperature}")
    if st != 0:
        raise RuntimeError(f"orc_search failed: {st}")
    out = dict(visits=visits, rootQ=rootQ, mm_max=mm[:, 0], mm_min=mm[:, 1], extra_ties=et,
               action=action, pi=pi, latent=latent, latent_len=latent_len, sel_steps=steps)
    if depths:
        out["depths"] = dep
    return out
