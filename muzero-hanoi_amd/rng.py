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

Any further tie the kernel meets is counted in `extra_ties` (none was observed in the
reference traces, tests/golden/rng_order.json); when it is non-zero the RNG streams of the two
implementations have diverged and the caller is told so.
"""
import numpy as np


def uses_noise(deterministic, alpha, eps):
    return (not deterministic) and alpha > 0.0 and eps > 0.0


def predraw(n_roots, *, deterministic, alpha, eps=0.25, rng=None, draw_action=True):
    """Draw (noise[B,6] f64 | None, tie[B] i32, u[B] f64 | None) from `rng` (default: the
    global legacy NumPy stream, exactly as the reference consumes it).  draw_action=False: a
    search that raises before its action draw (invalid temperature, mcts.py:113,163-166)."""
    rs = np.random if rng is None else rng
    noise = np.empty((n_roots, 6), np.float64) if uses_noise(deterministic, alpha, eps) else None
    tie = np.empty(n_roots, np.int32)
    u = None if (deterministic or not draw_action) else np.empty(n_roots, np.float64)
    alphas = np.ones(6, np.float32) * alpha  # np.ones_like(prob) * alpha with prob float32
    cand = np.arange(6)
    for r in range(n_roots):
        if noise is not None:
            noise[r] = rs.dirichlet(alphas)
        tie[r] = rs.choice(cand)
        if u is not None:
            u[r] = rs.random_sample()
    return noise, tie, u


def synthetic_draws(n_roots, *, deterministic, alpha, eps=0.25, seed=0):
    """Vectorised draws of the same distributions for large synthetic batches (bench).
    Not stream-compatible with the legacy global RNG; used where no parity claim is made."""
    g = np.random.default_rng(seed)
    noise = None
    if uses_noise(deterministic, alpha, eps):
        noise = g.dirichlet(np.full(6, np.float64(np.float32(alpha))), size=n_roots)
    tie = g.integers(0, 6, size=n_roots, dtype=np.int32)
    u = None if deterministic else g.random(n_roots)
    return noise, tie, u
