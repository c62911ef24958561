"""Host-side random draws, consumed in the reference's order.

The reference draws from NumPy's global legacy MT19937 stream inside `run_mcts`
(MCTS/mcts.py:57-66,149 Dirichlet; MCTS/node.py:86 argmax-tie choice; MCTS/mcts.py:118-120
action sample). The device search cannot call NumPy, so the host draws everything a batch of
`B` sequential `run_mcts` calls would draw, in the same order, and hands the results to the
kernel:

  per root r:  [noise_r  = dirichlet(ones(6, f32) * alpha)]   if stochastic and alpha>0 and eps>0
                tie_r    = choice(arange(6))                   the root's first selection is
                                                               always a 6-way tie (N_root = 0 =>
                                                               U = 0, Q = 0; README.md:49)
               [u_r      = random_sample()]                    if stochastic: choice(6, p=pi)

`predraw` makes those draws with libmzh's host restatement of NumPy's legacy algorithms
(`mzh_rng_predraw`, csrc/mzh_rng.cpp) on the RandomState's own MT19937 state, advanced in place
through the bit generator's ctypes interface: the same arrays and the same stream position as the
NumPy calls (`predraw_numpy`, kept as the specification and for RandomStates over another bit
generator), at C speed (65,536 roots: ~30 ms instead of ~1.3 s).

Any further tie the kernel meets is counted in `extra_ties` (none was observed in the
reference traces, tests/golden/rng_order.json); when it is non-zero the RNG streams of the two
implementations have diverged and the caller is told so.
"""
import ctypes

import numpy as np


def uses_noise(deterministic, alpha, eps):
    return (not deterministic) and alpha > 0.0 and eps > 0.0


def _alphas(alpha):
    """np.ones_like(prob) * alpha with prob float32 (mcts.py:148): float32 parameters"""
    return np.ones(6, np.float32) * alpha


def predraw_numpy(n_roots, *, deterministic, alpha, eps=0.25, rng=None, draw_action=True):
    """The reference's NumPy calls, one root at a time (the specification `predraw` restates)."""
    rs = np.random if rng is None else rng
    noise = np.empty((n_roots, 6), np.float64) if uses_noise(deterministic, alpha, eps) else None
    tie = np.empty(n_roots, np.int32)
    u = None if (deterministic or not draw_action) else np.empty(n_roots, np.float64)
    alphas = _alphas(alpha)
    cand = np.arange(6)
    for r in range(n_roots):
        if noise is not None:
            noise[r] = rs.dirichlet(alphas)
        tie[r] = rs.choice(cand)
        if u is not None:
            u[r] = rs.random_sample()
    return noise, tie, u


def _random_state(rng):
    rs = np.random.mtrand._rand if rng is None or rng is np.random else rng
    if not isinstance(rs, np.random.RandomState):
        raise TypeError(f"predraw needs a legacy numpy.random.RandomState (the reference's stream), got {type(rs)}")
    return rs


_CHECKED = False


def _self_check():
    """Once per process: the C restatement against NumPy on a private RandomState (a NumPy whose
    MT19937 state layout or legacy algorithms differed would fail here, loudly)."""
    global _CHECKED
    if _CHECKED:
        return
    for alpha, det in ((0.25, False), (2.5, False), (0.25, True)):
        a, b = np.random.RandomState(20261018), np.random.RandomState(20261018)
        got = _predraw_c(a, 16, deterministic=det, alpha=alpha, eps=0.25, draw_action=True)
        want = predraw_numpy(16, deterministic=det, alpha=alpha, rng=b)
        sa, sb = a.get_state(), b.get_state()
        same = all((x is None and y is None) or np.array_equal(x, y) for x, y in zip(got, want))
        if not (same and np.array_equal(sa[1], sb[1]) and sa[2:] == sb[2:]):
            raise RuntimeError("mzh_rng_predraw disagrees with this NumPy's legacy RandomState draws")
    _CHECKED = True


def _predraw_c(rs, n_roots, *, deterministic, alpha, eps, draw_action):
    from . import _lib

    L = _lib.lib()
    noisy = uses_noise(deterministic, alpha, eps)
    alphas = _alphas(alpha).astype(np.float64)
    if noisy and not (alphas > 0).all():
        raise ValueError("alpha <= 0")  # RandomState.dirichlet (alpha underflows in float32)
    noise = np.empty((n_roots, 6), np.float64) if noisy else None
    tie = np.empty(n_roots, np.int32)
    u = np.empty(n_roots, np.float64) if (not deterministic and draw_action) else None
    # the gamma sampler uses the polar Gaussian (and the RandomState's cached deviate) only for alpha > 1
    gauss_used = noisy and float(alphas[0]) > 1.0
    p = lambda x: None if x is None else x.ctypes.data_as(ctypes.c_void_p)
    # the bit generator's own lock (every RandomState method takes it): a NumPy draw on the same stream
    # from another thread cannot interleave with the in-place C loop
    with rs._bit_generator.lock:
        if gauss_used:
            st = rs.get_state()
            g = np.array([float(st[3]), st[4]], np.float64)
        else:
            g = np.zeros(2, np.float64)
        addr = rs._bit_generator.ctypes.state_address
        status = L.mzh_rng_predraw(ctypes.c_void_p(addr), p(g), int(n_roots), 6 if noisy else 0, p(alphas), 6,
                                   1 if u is not None else 0, p(noise), p(tie), p(u))
        _lib.check(status, "mzh_rng_predraw")
        if gauss_used:
            st = rs.get_state()  # the key / pos the C code advanced in place, with the new Gaussian cache
            rs.set_state((st[0], st[1], st[2], int(g[0]), float(g[1])))
    return noise, tie, u


_ALPHAS = {}
_STATE_ADDR = {}


def predraw_into(noise, tie, u, *, deterministic, alpha, eps=0.25, draw_action=True, addrs=None):
    """`predraw` for the one-root drop-in (MCTS.run_mcts, once per environment step) from the global legacy
    stream, written straight into the caller's arrays (numpy views of the pinned staging buffer): noise [1,6]
    f64, tie [1] i32, u [1] f64 -- each drawn only where `predraw` would draw it, the others left untouched.
    The same C restatement and the same lock; the per-call Python work (allocations, pointer conversions, the
    bit generator's state address) is cached.  addrs: the three arrays' data addresses, if the caller keeps them.
    Returns (noise drawn, u drawn)."""
    rs = np.random.mtrand._rand
    bg = rs._bit_generator
    if type(bg).__name__ != "MT19937":
        n2, t2, u2 = predraw(1, deterministic=deterministic, alpha=alpha, eps=eps, draw_action=draw_action)
        tie[...] = t2
        if n2 is not None:
            noise[...] = n2
        if u2 is not None:
            u[...] = u2
        return n2 is not None, u2 is not None
    _self_check()
    from . import _lib

    noisy = uses_noise(deterministic, alpha, eps)
    draw_u = not deterministic and draw_action
    key = float(alpha)
    al = _ALPHAS.get(key)
    if al is None:
        al = _alphas(alpha).astype(np.float64)
        _ALPHAS[key] = al
    if noisy and (not (al > 0).all() or float(al[0]) > 1.0):
        # alpha <= 0 raises like RandomState.dirichlet; alpha > 1 needs the Gaussian cache: the general path
        n2, t2, u2 = predraw(1, deterministic=deterministic, alpha=alpha, eps=eps, draw_action=draw_action)
        tie[...] = t2
        noise[...] = n2
        if u2 is not None:
            u[...] = u2
        return True, u2 is not None
    ent = _STATE_ADDR.get(id(bg))
    if ent is None or ent[0] is not bg:
        ent = (bg, bg.ctypes.state_address, np.zeros(2, np.float64))
        _STATE_ADDR[id(bg)] = ent
    na, ta, ua = addrs if addrs is not None else (noise.ctypes.data, tie.ctypes.data, u.ctypes.data)
    with bg.lock:
        st = _lib.lib().mzh_rng_predraw(ent[1], ent[2].ctypes.data, 1, 6 if noisy else 0, al.ctypes.data, 6,
                                        1 if draw_u else 0, na if noisy else None, ta, ua if draw_u else None)
    _lib.check(st, "mzh_rng_predraw")
    return noisy, draw_u


def predraw(n_roots, *, deterministic, alpha, eps=0.25, rng=None, draw_action=True):
    """Draw (noise[B,6] f64 | None, tie[B] i32, u[B] f64 | None) from `rng` (default: the global
    legacy NumPy stream), exactly as B sequential run_mcts calls consume it.  draw_action=False: a
    search that raises before its action draw (invalid temperature, mcts.py:113,163-166)."""
    rs = _random_state(rng)
    if type(rs._bit_generator).__name__ != "MT19937":
        return predraw_numpy(n_roots, deterministic=deterministic, alpha=alpha, eps=eps, rng=rs,
                             draw_action=draw_action)
    _self_check()
    return _predraw_c(rs, n_roots, deterministic=deterministic, alpha=alpha, eps=eps, draw_action=draw_action)


def synthetic_draws(n_roots, *, deterministic, alpha, eps=0.25, seed=0):
    """Vectorised draws of the same distributions for large synthetic batches.
    Not stream-compatible with the legacy global RNG; used where no parity claim is made.
    Each quantity comes from its own child stream of `seed`, so the draws for n roots are the first n rows of
    the draws for any larger count (BatchedSelfPlay draws a move's batch before it knows how many envs are left)."""
    gn, gt, gu = (np.random.default_rng(s) for s in np.random.SeedSequence(seed).spawn(3))
    noise = None
    if uses_noise(deterministic, alpha, eps):
        noise = gn.dirichlet(np.full(6, np.float64(np.float32(alpha))), size=n_roots)
    tie = gt.integers(0, 6, size=n_roots, dtype=np.int32)
    u = None if deterministic else gu.random(n_roots)
    return noise, tie, u
