"""rng.predraw (libmzh's host restatement of NumPy's legacy draws, csrc/mzh_rng.cpp) against
NumPy's own RandomState calls (rng.predraw_numpy: MCTS/mcts.py:57-66,149 Dirichlet, MCTS/node.py:86
tie choice, MCTS/mcts.py:118-120 action sample): identical arrays and identical stream state
afterwards, at the bench's full 65,536-root batch.  CPU only (host code; no device needed)."""
import time

import numpy as np
import pytest


@pytest.fixture(scope="module")
def rng():
    from muzero_hanoi_amd import build

    build.build()
    from muzero_hanoi_amd import rng as mrng

    return mrng


def _same_state(a, b):
    sa, sb = a.get_state(), b.get_state()
    return np.array_equal(sa[1], sb[1]) and sa[2:] == sb[2:]


def _same(x, y):
    return all((p is None and q is None) or (p is not None and q is not None and np.array_equal(p, q))
               for p, q in zip(x, y))


@pytest.mark.parametrize("alpha", [0.0, 0.25, 0.3])
@pytest.mark.parametrize("deterministic", [False, True])
def test_predraw_equals_numpy_65536_roots(rng, alpha, deterministic):
    a, b = np.random.RandomState(11), np.random.RandomState(11)
    got = rng.predraw(65536, deterministic=deterministic, alpha=alpha, rng=a)
    want = rng.predraw_numpy(65536, deterministic=deterministic, alpha=alpha, rng=b)
    assert _same(got, want)
    assert _same_state(a, b)
    # and the streams stay in step afterwards
    assert np.array_equal(a.random_sample(8), b.random_sample(8))


def test_predraw_global_stream(rng):
    """default rng = the reference's global np.random stream, advanced in place"""
    np.random.seed(5)
    got = rng.predraw(3000, deterministic=False, alpha=0.25)
    after = np.random.get_state()
    np.random.seed(5)
    want = rng.predraw_numpy(3000, deterministic=False, alpha=0.25)
    assert _same(got, want)
    now = np.random.get_state()
    assert np.array_equal(after[1], now[1]) and after[2:] == now[2:]


@pytest.mark.parametrize("alpha", [1.0, 2.5])
def test_predraw_gamma_branches(rng, alpha):
    """alpha == 1 (the exponential branch) and alpha > 1 (Marsaglia-Tsang on the polar Gaussian,
    whose cached second deviate is part of the RandomState's state), including a Gaussian cached
    before the call"""
    a, b = np.random.RandomState(3), np.random.RandomState(3)
    a.standard_normal()
    b.standard_normal()  # leaves has_gauss = 1
    got = rng.predraw(4000, deterministic=False, alpha=alpha, rng=a)
    want = rng.predraw_numpy(4000, deterministic=False, alpha=alpha, rng=b)
    assert _same(got, want)
    assert _same_state(a, b)
    assert a.standard_normal() == b.standard_normal()


def test_predraw_without_action_draw(rng):
    """a search that raises before its action draw (bad temperature, mcts.py:113,163-166)"""
    a, b = np.random.RandomState(9), np.random.RandomState(9)
    got = rng.predraw(500, deterministic=False, alpha=0.25, rng=a, draw_action=False)
    want = rng.predraw_numpy(500, deterministic=False, alpha=0.25, rng=b, draw_action=False)
    assert got[2] is None and _same(got, want) and _same_state(a, b)


def test_predraw_stream_wraps_many_times(rng):
    """pos at every offset of the 624-word key: batches of 1..40 roots back to back"""
    a, b = np.random.RandomState(123), np.random.RandomState(123)
    for n in range(1, 41):
        got = rng.predraw(n, deterministic=(n % 3 == 0), alpha=0.25, rng=a)
        want = rng.predraw_numpy(n, deterministic=(n % 3 == 0), alpha=0.25, rng=b)
        assert _same(got, want), n
    assert _same_state(a, b)


def test_predraw_rejects_float32_zero_alpha(rng):
    """alpha > 0 that rounds to 0 in float32: NumPy's dirichlet raises ValueError('alpha <= 0')"""
    a, b = np.random.RandomState(1), np.random.RandomState(1)
    with pytest.raises(ValueError):
        rng.predraw_numpy(1, deterministic=False, alpha=1e-60, rng=b)
    with pytest.raises(ValueError):
        rng.predraw(1, deterministic=False, alpha=1e-60, rng=a)
    assert _same_state(a, b)


def test_predraw_speed(rng):
    """the headline batch's reference-order draws at C speed (<= 30 ms for 65,536 roots;
    the bound here is loose because shared CI hosts vary, the bench line records the real figure)"""
    rs = np.random.RandomState(0)
    rng.predraw(1024, deterministic=False, alpha=0.25, rng=rs)
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        rng.predraw(65536, deterministic=False, alpha=0.25, rng=rs)
        best = min(best, time.perf_counter() - t0)
    assert best < 0.1, best
