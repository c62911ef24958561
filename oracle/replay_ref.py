"""Restatement of the device replay draw (csrc/mzh_replay.hip) -- TEST INFRASTRUCTURE ONLY.

The reference's prioritised draw (buffer.py:89-112) is NumPy: P = p / np.sum(p) in float32, then
np.random.choice(np.arange(n), m, replace=True, p=P), which RandomState computes as a float64 cumsum
of P, divided by its last entry, searched with searchsorted(u, 'right') for m uniforms u.  The device
kernel restates both sums in another shape; this module restates the kernel's algorithm step by step
in NumPy so that tests/test_replay.py can pin it on the CPU against NumPy itself:
  * `numpy_f32_sum`: np.sum over a float32 array as NumPy 2.x computes it (0 + the pairwise sums of
    consecutive 8,192-element buffers; a buffer's pairwise sum splits n at n/2 rounded down to a
    multiple of 8 until a block has <= 128 elements, summed with 8 interleaved accumulators);
  * `exact_cumsum_applies` / `scan_cdf`: when every non-zero probability is >= 2^-28 and the total
    is below 4, every partial sum is a multiple of 2^-51 below 4 (an exact float64 value), so the
    workgroup's float64 scan of segment sums equals the sequential chain (restated here as an
    integer scan in units of 2^-51);
  * `draw`: the whole draw (validity, cdf, the 4,096-entry sample search) -> indices.
"""
import numpy as np

CHUNK, BLOCK, NC = 8192, 128, 4096
UNIT = 2.0 ** 51
MIN_EXACT = np.float32(2.0 ** -28)


def _block_sum(a):
    n = len(a)
    if n < 8:
        r = np.float32(0)
        for x in a:
            r = np.float32(r + x)
        return r
    r = [np.float32(a[j]) for j in range(8)]
    n8 = n - n % 8
    for i in range(8, n8, 8):
        for j in range(8):
            r[j] = np.float32(r[j] + a[i + j])
    res = np.float32(np.float32(np.float32(r[0] + r[1]) + np.float32(r[2] + r[3]))
                     + np.float32(np.float32(r[4] + r[5]) + np.float32(r[6] + r[7])))
    for i in range(n8, n):
        res = np.float32(res + a[i])
    return res


def _pairwise(a):
    n = len(a)
    if n <= BLOCK:
        return _block_sum(a)
    h = n // 2
    h -= h % 8
    return np.float32(_pairwise(a[:h]) + _pairwise(a[h:]))


def numpy_f32_sum(a):
    a = np.asarray(a, np.float32)
    s = np.float32(0)
    for c in range(0, len(a), CHUNK):
        s = np.float32(s + _pairwise(a[c:c + CHUNK]))
    return s


def exact_cumsum_applies(probs):
    q = np.asarray(probs, np.float32)
    nz = q[q != 0]
    if len(nz) and nz.min() < MIN_EXACT:
        return False
    return int((q.astype(np.float64) * UNIT).astype(np.int64).sum()) < 2 ** 53


def scan_cdf(probs):
    """the kernel's exact path: integer prefix sums of P_i * 2^51, back to float64"""
    v = (np.asarray(probs, np.float32).astype(np.float64) * UNIT).astype(np.int64)
    return np.cumsum(v).astype(np.float64) / UNIT


def draw(prio, u):
    """indices the kernel returns for priorities `prio` (float32) and uniforms `u` (float64), or None
    where NumPy's choice raises (a NaN or negative probability)"""
    p = np.asarray(prio, np.float32)
    n = len(p)
    probs = p / numpy_f32_sum(p)
    if not np.all((probs >= 0) & (probs <= 1)):
        return None
    cdf = scan_cdf(probs) if exact_cumsum_applies(probs) else probs.astype(np.float64).cumsum()
    last = cdf[-1]
    stride = (n + NC - 1) // NC
    nc = (n + stride - 1) // stride
    sample = cdf[np.minimum(n, (np.arange(nc) + 1) * stride) - 1] / last
    out = np.empty(len(u), np.int64)
    for k, uk in enumerate(np.asarray(u, np.float64)):
        j = int(np.searchsorted(sample, uk, side="right"))
        lo, hi = j * stride, min(n, (j + 1) * stride) - 1
        while lo < hi:
            mid = (lo + hi) // 2
            if cdf[mid] / last > uk:
                hi = mid
            else:
                lo = mid + 1
        out[k] = lo
    return out
