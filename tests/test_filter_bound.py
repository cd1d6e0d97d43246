"""The bf16 filter's error bound (tt_filter.hip header, k_query_eps) -- CPU checks.

The filter keeps every row whose bf16 score a lies within 2*eps_q of the bf16 k-th best, so
exactness rests on |a - s| <= eps_q for every (row, query).  Here the rounding part of the
bound is checked in float64 against emulated bf16 round-to-nearest-even, on random and on
adversarial inputs (every component rounding the same way), and the worst-case-u bound this
replaced is shown to be violated by the adversarial case.
"""
import numpy as np


def bf16_rne(x):
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32)


def rounding_bound(X, R, q):
    """R|q| + (X+R)|q - q~|: the Cauchy-Schwarz part of eps_q (accumulation terms aside)."""
    qt = bf16_rne(q).astype(np.float64)
    return R * np.linalg.norm(q) + (X + R) * np.linalg.norm(q - qt)


def check(x, q):
    x = x.astype(np.float32)
    q = q.astype(np.float32)
    xt = bf16_rne(x).astype(np.float64)
    X = np.linalg.norm(x.astype(np.float64), axis=1).max()
    R = np.linalg.norm(x - xt, axis=1).max()
    err = np.abs(x.astype(np.float64) @ q.astype(np.float64) - xt @ bf16_rne(q).astype(np.float64))
    return err, rounding_bound(X, R, q.astype(np.float64))


def test_bound_holds_on_random_rows():
    rng = np.random.default_rng(0)
    x = rng.standard_normal((20000, 384))
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    for _ in range(5):
        q = rng.standard_normal(384)
        q /= np.linalg.norm(q)
        err, b = check(x, q)
        assert err.max() <= b
        assert b < 2.0 ** -8  # measured residuals: tighter than the worst case


def test_bound_holds_on_adversarial_rounding():
    # every component just above a rounding midpoint: all round up by ~2^-8 relative
    d = 384
    v = np.float32(2.0 ** -5 * (1 + 2.0 ** -8 + 2.0 ** -20))  # mantissa just past a midpoint
    x = np.full((1, d), v, np.float32)
    q = np.full(d, v, np.float32)
    err, b = check(x, q)
    assert err.max() <= b
    # the previous bound (2^-8 + 2^-18) |x||q| does NOT cover this case
    old = (2.0 ** -8 + 2.0 ** -18) * np.linalg.norm(x) * np.linalg.norm(q)
    assert err.max() > old
