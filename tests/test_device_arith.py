"""Host restatements of the device-side integer shortcuts, checked against the exact operation.

`mod_f64` (csrc/ransac.hip) replaces OpenCV's `RNG::uniform(0, n) = next() % n`
(operations.hpp, called from getSubset in ptsetreg.cpp) in the attempt kernel: floor(a * fl(1/n))
on the fp64 pipe, exact remainder, one correction.  numpy float64 follows the same IEEE rounding
(q * n < 2^33 is exact, so the device's fma and the plain multiply-subtract agree).
"""
import numpy as np


def mod_f64(a, n):
    a = a.astype(np.float64)
    nf = np.float64(n)
    inv = np.float64(1.0) / nf
    r = a - np.floor(a * inv) * nf
    r = np.where(r < 0, r + nf, r)
    r = np.where(r >= nf, r - nf, r)
    return r.astype(np.uint64)


def test_mod_f64_exact_random():
    rng = np.random.default_rng(7)
    for n in [5, 7, 1999, 2000, 2048, 10000, 50000, 65535, 65537, 999983, (1 << 24) + 1, (1 << 31) - 1]:
        a = rng.integers(0, 1 << 32, size=400_000, dtype=np.uint64)
        assert np.array_equal(mod_f64(a, n), a % np.uint64(n)), n


def test_mod_f64_exact_near_multiples():
    # quotient boundaries are where floor(a * fl(1/n)) can be off by one
    for n in [3, 1999, 2000, 40961, 65535, 1234567, (1 << 31) - 1]:
        k = np.arange(0, (1 << 32) // n + 1, max(1, ((1 << 32) // n) // 50_000), dtype=np.uint64)
        base = k * np.uint64(n)
        a = np.concatenate([base, base + np.uint64(1), np.where(base > 0, base - np.uint64(1), base),
                            np.array([(1 << 32) - 1], dtype=np.uint64)])
        a = a[a < (1 << 32)]
        assert np.array_equal(mod_f64(a, n), a % np.uint64(n)), n
