"""Host restatements of the device-side integer shortcuts, checked against the exact operation.

`mod_barrett` (csrc/ransac.hip) replaces OpenCV's `RNG::uniform(0, n) = next() % n`
(operations.hpp, called from getSubset in ptsetreg.cpp) in the attempt kernel:
q = mulhi(a, floor((2^32-1)/n)), r = a - q*n in [0, 2n), r = min(r, r - n) as uint32.
"""
import numpy as np


def mod_barrett(a, n):
    a = a.astype(np.uint64)
    m = np.uint64((2**32 - 1) // n)
    q = (a * m) >> np.uint64(32)
    r = (a - q * np.uint64(n)) & np.uint64(0xFFFFFFFF)
    r2 = (r - np.uint64(n)) & np.uint64(0xFFFFFFFF)
    return np.minimum(r, r2)


NS = [1, 2, 3, 5, 7, 255, 256, 257, 1999, 2000, 2048, 10000, 50000, 65535, 65537, 999983, (1 << 24) + 1,
      (1 << 31) - 1, (1 << 31), (1 << 32) - 1]


def test_mod_barrett_exact_random():
    rng = np.random.default_rng(7)
    for n in NS:
        a = rng.integers(0, 1 << 32, size=400_000, dtype=np.uint64)
        assert np.array_equal(mod_barrett(a, n), a % np.uint64(n)), n


def test_mod_barrett_exact_near_multiples():
    # quotient boundaries are where mulhi(a, m) falls one short
    for n in NS:
        step = max(1, ((1 << 32) // n) // 50_000)
        k = np.arange(0, (1 << 32) // n + 1, step, dtype=np.uint64)
        base = k * np.uint64(n)
        a = np.concatenate([base, base + np.uint64(1), np.where(base > 0, base - np.uint64(1), base),
                            np.array([(1 << 32) - 1, (1 << 32) - 2], dtype=np.uint64)])
        a = a[a < (1 << 32)]
        assert np.array_equal(mod_barrett(a, n), a % np.uint64(n)), n


def test_q_times_n_fits_24_bits_above_256():
    # the device uses v_mul_u32_u24 for q*n when n > 256: q < 2^24 and n < 2^24 there
    for n in [257, 2000, 65535, (1 << 24) - 1]:
        assert ((2**32 - 1) // n) < (1 << 24)


def fastmod_from_M(a, n):
    """csrc/ransac.hip fastmod: Barrett with m = M >> 32, M = floor((2^64-1)/n) + 1 (RansacState::modM)."""
    a = a.astype(np.uint64)
    M = ((2**64 - 1) // n + 1) % 2**64
    m = np.uint64(M >> 32)
    q = (a * m) >> np.uint64(32)
    r = (a - q * np.uint64(n)) & np.uint64(0xFFFFFFFF)
    r2 = (r - np.uint64(n)) & np.uint64(0xFFFFFFFF)
    return np.minimum(r, r2)


def test_fastmod_from_lemire_constant():
    rng = np.random.default_rng(11)
    for n in [2, 3, 4, 5, 1024, 1999, 2000, 4096, 65536, 65537, 999983, (1 << 31) - 1, 1 << 31, (1 << 32) - 1]:
        a = np.concatenate([rng.integers(0, 1 << 32, size=200_000, dtype=np.uint64),
                            np.array([0, 1, n - 1, n, n + 1, (1 << 32) - 1], dtype=np.uint64) % np.uint64(1 << 32)])
        assert np.array_equal(fastmod_from_M(a, n), a % np.uint64(n)), n


# ------------------------------------------------------------------------------------------------
# Early tiles of knn2_i8_kernel (csrc/knn.hip tile_early): a value R = q'.t'' + floor(n2/2) of train
# row `row` (0..63 within its tile, n2 & 1 = p) becomes the 32-bit key (R << 8) + K, K = 2^28 + 128 p +
# row (prep_tile's norm words 192..255), so that unsigned key order is (D, row) order with
# D = 2R + p = d^2 - c(q), decoded as D = (key - 2^28) >> 7 (arithmetic), row = key & 127.  Padded rows
# (R = 2^30 - 1 exactly, t'' = 0; K = 255) wrap to UINT_MAX and never enter the top-2.
# ------------------------------------------------------------------------------------------------
def early_key(R, p, row):
    K = (1 << 28) + 128 * p.astype(np.int64) + row.astype(np.int64)
    return ((R.astype(np.int64) << 8) + K) & 0xFFFFFFFF


def d_range():
    # D = d^2 - c(q), c(q) = |q - 128|^2 + 2 sum(q - 128) = sum((q - 127)^2 - 1), q, t in [0, 255]^128
    d2_max = 128 * 255 * 255
    c_max = 128 * ((0 - 127) ** 2 - 1)
    c_min = -128
    return -c_max, d2_max - c_min


def test_early_key_order_and_decode():
    rng = np.random.default_rng(11)
    dlo, dhi = d_range()
    D = np.concatenate([rng.integers(dlo, dhi + 1, 300_000), np.array([dlo, dhi, 0, -1, 1]),
                        rng.integers(-50, 50, 100_000)])  # many equal D: the row decides
    row = rng.integers(0, 64, D.size)
    p = D & 1
    R = (D - p) >> 1  # floor((D - p) / 2): D = 2R + p
    key = early_key(R, p, row)
    assert key.min() > 0 and key.max() < (1 << 31), "real keys stay in (0, 2^31)"
    # decode
    k32 = key.astype(np.int64)
    assert np.array_equal((k32 - (1 << 28)) >> 7, D)
    assert np.array_equal(k32 & 127, row)
    # unsigned key order == lexicographic (D, row) order
    o_key = np.argsort(key, kind="stable")
    o_lex = np.lexsort((row, D))
    assert np.array_equal(key[o_key], key[o_lex])


def test_early_key_padded_row_is_uint_max():
    R = np.array([(1 << 30) - 1])
    K = 255
    assert ((int(R[0]) << 8) + K) & 0xFFFFFFFF == 0xFFFFFFFF

