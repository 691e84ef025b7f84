"""The correctly rounded exp shared by the HIP Bratu stencils and the oracle (csrc/nk_exp.h), pinned on CPU.

Every Bratu residual / JVP / FD value goes through this one function on both sides
(examples/bratu.jl:21's lam * exp(u)), which is what makes the Bratu path bit-identical to the oracle.
Here it is checked independently of both: against mpmath at 250 bits rounded once to binary64
(tests/golden/make_exp_golden.py's cr_exp), on >= 10^6 inputs over the Bratu range, the whole finite
range, the subnormal and overflow bands and inputs built to defeat the fast phase's Ziv test; and
against the reference's own known answer exp(2.0) == 7.38905609893065 (test/runtests.jl:38).
"""
import os
import re
import sys

import mpmath
import numpy as np
import pytest

import _nkpath  # noqa: F401
from oracle import oracle as oc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import gen_exp_consts as gen  # noqa: E402
from make_exp_golden import cr_exp  # noqa: E402

HDR = os.path.join(ROOT, "newtonkrylov.jl_amd", "csrc", "nk_exp.h")


def same(a, b):
    return (a == b) | (np.isnan(a) & np.isnan(b))


def test_reference_known_answer():
    """test/runtests.jl:36-38: mul!(out, J, [1, 0]) == [6.0, 7.38905609893065], i.e. exp(2.0) exactly."""
    assert oc.exp(np.array([2.0]))[0] == 7.38905609893065
    assert oc.exp(np.array([1.0]))[0] == 2.718281828459045


def test_special_values():
    x = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-300, -1e-300, 746.0, -746.0, 709.782712893384,
                  709.7827128933841, -745.1332191019411, -745.1332191019412])
    y = oc.exp(x)
    assert y[0] == 1.0 and y[1] == 1.0 and y[2] == np.inf and y[3] == 0.0 and np.isnan(y[4])
    assert y[5] == 1.0 and y[6] == 1.0 and y[7] == np.inf and y[8] == 0.0
    assert y[9] == 1.7976931348622732e308 and y[10] == np.inf  # the overflow threshold
    assert y[11] == 5e-324 and y[12] == 0.0  # the least subnormal and below


def test_golden_vectors(golden_dir):
    d = np.load(os.path.join(golden_dir, "exp_cr.npz"))
    assert np.all(same(oc.exp(d["x"]), d["y"]))


def test_constants_match_generator():
    """Every constant in nk_exp.h is what tools/gen_exp_consts.py derives with mpmath."""
    src = open(HDR).read()
    h, m, l = gen.ln2n_split()
    c3, c4, c5, c6, c7 = gen.coeffs()
    for name, v in (("NKX_INVLN2N", gen.invln2n()), ("NKX_L2N_H", h), ("NKX_L2N_M", m), ("NKX_L2N_L", l),
                    ("NKX_C3", c3), ("NKX_C4", c4), ("NKX_C5", c5), ("NKX_C6", c6), ("NKX_C7", c7)):
        got = re.search(rf"#define {name} (\S+)", src).group(1)
        assert float.fromhex(got) == v, name
    tab = re.findall(r"\{(-?0x[0-9a-fp.+-]+), (-?0x[0-9a-fp.+-]+)\},\s+/\* (\d+) \*/", src)
    assert len(tab) == 128
    for (a, b, j), (hi, lo) in zip(tab, gen.table()):
        assert float.fromhex(a) == hi and float.fromhex(b) == lo, j
    ln2 = re.search(r"NKX_LN2_FX\[3\] = \{\s*(0x\w+)ULL, (0x\w+)ULL, (0x\w+)ULL", src).groups()
    assert [int(w, 16) for w in ln2] == gen.limbs(gen.ln2_fx())
    fac = re.findall(r"\{(0x\w+)ULL, (0x\w+)ULL, (0x\w+)ULL\},\s+/\* 1/(\d+)! \*/", src)
    assert len(fac) == 18
    for (a, b, c, i), v in zip(fac, gen.invfact_fx()):
        assert [int(a, 16), int(b, 16), int(c, 16)] == gen.limbs(v), i


def _mp_exp(x):
    return np.array([cr_exp(v) for v in x])


def test_correctly_rounded_million():
    """10^6 inputs over the Bratu range (u + eps v in [-1, 3]) plus 2 x 10^5 over the finite range: every
    result equals mpmath's correctly rounded value."""
    rng = np.random.default_rng(7)
    x = np.concatenate([rng.uniform(-1.0, 3.0, 1_000_000), rng.uniform(-708.0, 709.7, 100_000),
                        rng.uniform(-745.2, -708.2, 50_000), rng.uniform(709.77, 709.8, 10_000),
                        rng.choice([-1.0, 1.0], 40_000) * 2.0 ** rng.uniform(-60, -3, 40_000)])
    y = oc.exp(x)
    ref = _mp_exp(x)
    bad = ~same(y, ref)
    assert not bad.any(), (x[bad][:5], y[bad][:5], ref[bad][:5])


def test_exact_phase_alone():
    """The fixed-point phase on its own (not only where the Ziv test sends it) is correctly rounded."""
    rng = np.random.default_rng(8)
    x = np.concatenate([rng.uniform(-1.0, 3.0, 30_000), rng.uniform(-745.0, 709.7, 30_000),
                        rng.choice([-1.0, 1.0], 10_000) * 2.0 ** rng.uniform(-53, -3, 10_000)])
    assert np.all(oc.exp_slow(x) == _mp_exp(x))


def test_ziv_cases_take_the_exact_phase():
    """Inputs whose exp lies within ~2^-73 of a rounding midpoint: the fast phase alone cannot decide
    them, the Ziv test hands them over, and the result is still the correctly rounded one."""
    a = np.arange(2 ** 16, 2 ** 16 + 3000, dtype=np.float64)
    x = np.concatenate([a * 2.0 ** -52 + 2.0 ** -53, -(a * 2.0 ** -52 + 2.0 ** -53)])
    _, _, _, slow = oc.exp_dd(x)
    assert slow > len(x) // 10
    assert np.all(oc.exp(x) == _mp_exp(x))


def test_fast_phase_error_bound():
    """The fast phase's double-double result is within 2^-76 (relative) of exp(x) -- the bound DESIGN.md
    §2 derives; the Ziv test is valid up to 2^-73 (measured ~2^-79).  Random inputs over the Bratu and the
    finite range, plus the reduction's hard cases: x next to a multiple k ln2/128 (r ~ 0) and x at a
    half step (|r| maximal), with |k| up to 2^17."""
    rng = np.random.default_rng(9)
    L = np.log(2) / 128
    k = rng.integers(-130_000, 130_000, 3000)
    x = np.concatenate([rng.uniform(-1.0, 3.0, 3000), rng.uniform(-708.0, 709.7, 3000),
                        k * L + rng.uniform(-1e-12, 1e-12, 3000) * L, (k + 0.5) * L])
    x = x[(x > -708.3) & (x < 709.78)]
    zh, zl, m, _ = oc.exp_dd(x)
    mpmath.mp.prec = 250
    worst = mpmath.mpf(0)
    for xi, a, b, k in zip(x, zh, zl, m):
        e = mpmath.exp(mpmath.mpf(float(xi))) / mpmath.ldexp(1, int(k))
        worst = max(worst, abs((mpmath.mpf(float(a)) + mpmath.mpf(float(b)) - e) / e))
    assert worst < mpmath.ldexp(1, -76), float(mpmath.log(worst, 2))


@pytest.mark.parametrize("lo,hi", [(-1.0, 3.0), (-700.0, 700.0)])
def test_ziv_rate(lo, hi):
    """The exact phase runs for ~2^-18 of random inputs (it costs the stencils nothing measurable)."""
    x = np.random.default_rng(10).uniform(lo, hi, 1_000_000)
    _, _, _, slow = oc.exp_dd(x)
    assert slow <= 40
