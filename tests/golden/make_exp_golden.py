"""Golden vectors of the correctly rounded exp (csrc/nk_exp.h) -> tests/golden/exp_cr.npz.

The expected outputs come from mpmath at 250 bits, rounded once to binary64 (subnormals by integer
rounding of exp(x) 2^1074, so no double rounding).  Inputs: the reference's own known answer
exp(2.0) == 7.38905609893065 (test/runtests.jl:38, the JVP's e^2), special values, the Bratu range,
the whole finite range, the subnormal and overflow bands, and near-midpoint inputs that defeat the fast
phase's Ziv test (x = a 2^-52 + 2^-53 with |x| ~ 2^-36: 1 + x is a midpoint and x^2/2 ~ 2^-73 decides).

    python tests/golden/make_exp_golden.py        (deterministic: numpy default_rng(2026))
"""
import os

import mpmath
import numpy as np

mpmath.mp.prec = 250
HERE = os.path.dirname(os.path.abspath(__file__))


def cr_exp(x: float) -> float:
    """exp(x) correctly rounded to binary64 (round to nearest even)."""
    if np.isnan(x):
        return float("nan")
    if x == float("inf"):
        return float("inf")
    if x == float("-inf"):
        return 0.0
    v = mpmath.exp(mpmath.mpf(float(x)))
    if v >= mpmath.ldexp(1, 1024) * (1 - mpmath.ldexp(1, -54)):
        return float("inf")
    if v < mpmath.ldexp(1, -1022):
        return float(int(mpmath.nint(mpmath.ldexp(v, 1074)))) * 2.0 ** -1074
    return float(v)


def inputs(seed=2026):
    rng = np.random.default_rng(seed)
    special = np.array([2.0, 1.0, -1.0, 0.0, -0.0, 0.5, 3.0, 1e-300, -1e-300, 2.0 ** -54, -(2.0 ** -54),
                        2.0 ** -53, 709.782712893384, 709.7827128933841, 709.79, -708.3, -708.39641853226408,
                        -745.1332191019411, -745.1332191019412, -745.14, -746.0, 746.0])
    a = rng.integers(2 ** 16, 2 ** 17, 2000).astype(np.float64)
    hard = a * 2.0 ** -52 + 2.0 ** -53
    return np.concatenate([
        special,
        rng.uniform(-1.0, 3.0, 3000),             # u + eps v of the Bratu stencils
        rng.uniform(-708.0, 709.7, 1000),
        rng.uniform(-745.2, -708.2, 500),         # subnormal results
        rng.uniform(709.77, 709.8, 200),          # overflow band
        rng.choice([-1.0, 1.0], 1000) * 2.0 ** rng.uniform(-60, -5, 1000),
        hard, -hard,
    ])


def main():
    x = inputs()
    y = np.array([cr_exp(v) for v in x])
    np.savez_compressed(os.path.join(HERE, "exp_cr.npz"), x=x, y=y)
    print(f"{len(x)} vectors -> exp_cr.npz")


if __name__ == "__main__":
    main()
