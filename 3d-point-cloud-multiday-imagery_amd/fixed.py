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
