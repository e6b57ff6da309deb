"""CPU check of the identities the device Jacobi rotation relies on (csrc/ransac.hip, jacobi_group and
jacobi_fast): OpenCV's JacobiImpl_ computes t = |y| + hypot(p, y), s = hypot(p, t) and p / t
(modules/core/src/lapack.cpp, as restated in oracle/mim_oracle.c); the kernels take hypot(p, t) as
t * sqrt(1 + q * q) with q = |p| / t and p / t as copysign(q, p).  Both are exact in IEEE doubles
because t >= |p| > 0, so hypot's larger operand is t, and division is sign-symmetric."""
import math

import numpy as np


def _hypot_cv(a: float, b: float) -> float:
    # OpenCV's hypot<double> (lapack.cpp), as oracle/mim_oracle.c and d_hypot restate it
    a, b = abs(a), abs(b)
    if a > b:
        r = b / a
        return a * math.sqrt(1 + r * r)
    if b > 0:
        r = a / b
        return b * math.sqrt(1 + r * r)
    return 0.0


def test_rotation_quotient_identities():
    rng = np.random.default_rng(7)
    n = 200_000
    scale = 10.0 ** rng.uniform(-12, 12, size=(n, 2))
    ps = rng.standard_normal(n) * scale[:, 0]
    ys = rng.standard_normal(n) * scale[:, 1]
    ys[::17] = 0.0  # y = 0: t == |p| exactly
    ys[1::17] = ps[1::17] * 0.5  # equal-magnitude neighbourhoods
    bad = 0
    for p, y in zip(ps.tolist(), ys.tolist()):
        if abs(p) <= 2.220446049250313e-16:
            continue
        t = abs(y) + _hypot_cv(p, y)
        assert t >= abs(p) > 0
        q = abs(p) / t
        bad += _hypot_cv(p, t) != t * math.sqrt(1 + q * q)
        bad += p / t != math.copysign(q, p)
    assert bad == 0
