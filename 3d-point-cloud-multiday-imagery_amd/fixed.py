"""Fixed-point scale of the exact centroid sums (product side).

Each coordinate enters the per-cluster sums as ``xq = trunc(ldexp(x, q_a))``
(exact power-of-two scaling, truncation toward zero) with ``q_a = QBITS - e_a``
where ``max|x_a| < 2**e_a`` over the WHOLE cloud (all ranks), so
``|xq| < 2**QBITS``.  The kernels keep per-lane partial sums of at most 63
points in int32 and every other sum in int64, which makes the centroid update
independent of summation order, block order and GPU count.
"""
from __future__ import annotations

import math

QBITS = 25


def fixed_q(maxabs) -> list:
    out = []
    for m in maxabs:
        m = float(m)
        e = 0 if m == 0.0 else math.frexp(m)[1]
        out.append(QBITS - e)
    return out


def inertia_from_limbs(limbs, scale: int, overflow: int = 0) -> float:
    """Global inertia from the (all-reduced) exact limbs of pcm_status:
    ``ldexp(float(l0 + l1 * 2**32 + l2 * 2**64), -scale)`` -- Python's int -> float
    conversion rounds once to nearest, like ``pcm_inertia_value``."""
    if overflow:
        return math.inf
    total = int(limbs[0]) + (int(limbs[1]) << 32) + (int(limbs[2]) << 64)
    return math.ldexp(float(total), -int(scale))
