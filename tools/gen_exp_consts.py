"""Generate the constants of the correctly rounded exp (newtonkrylov.jl_amd/csrc/nk_exp.h) with mpmath.

Prints C initialisers (hex-float doubles and 64-bit limbs); nk_exp.h holds their output verbatim, and
tests/test_exp.py re-derives every constant from this script's functions and compares.

  NKX_T[j] = (hi, lo)  2^(j/128) = hi + lo to ~107 bits, j = 0..127 (the fast path's table)
  L2N_H/M/L            ln2/128 = H + M + L, H with 21 significant bits (kd * H exact for |kd| < 2^32; a
                       double whose low 32 bits are zero, which gfx950's VOP2 fmac takes as a literal)
  INVLN2N              128/ln2 to 21 significant bits (k may then be off the nearest integer by one only
                       near a half: |r| <= 1.125 ln2/256, inside the fast phase's error analysis)
  C6, C7               1/720, 1/5040 to 21 significant bits (their terms are below 2^-60 and 2^-72)
  LN2_FX               round(ln2 * 2^190) as three 64-bit limbs (the slow path's fixed point, Q2.190)
  INVFACT_FX[i]        round(2^190 / i!), i = 0..17
"""
import mpmath

mpmath.mp.prec = 400
N = 128
FX = 190


def dbl(v):
    return float(v)  # mpmath rounds to nearest


def split_hi_lo(v):
    hi = dbl(v)
    lo = dbl(v - mpmath.mpf(hi))
    return hi, lo


def table():
    return [split_hi_lo(mpmath.power(2, mpmath.mpf(j) / N)) for j in range(N)]


def ln2n_split():
    c = mpmath.log(2) / N
    m, e = mpmath.frexp(c)  # c = m 2^e, 0.5 <= m < 1
    hi = mpmath.ldexp(mpmath.floor(mpmath.ldexp(m, 21)), e - 21)  # 21 significant bits
    h = float(hi)
    assert mpmath.mpf(h) == hi
    mid = dbl(c - hi)
    low = dbl(c - hi - mpmath.mpf(mid))
    return h, mid, low


def short21(v):
    """v rounded to 21 significant bits (the high 32-bit word of a double, the low word zero)"""
    m, e = mpmath.frexp(mpmath.mpf(v))
    return float(mpmath.ldexp(mpmath.nint(mpmath.ldexp(m, 21)), e - 21))


def invln2n():
    return short21(N / mpmath.log(2))


def coeffs():
    """C3 .. C7 of the cubic tail r^3 (C3 + r (C4 + r (C5 + r (C6 + r C7))))"""
    return [dbl(1 / mpmath.factorial(3)), dbl(1 / mpmath.factorial(4)), dbl(1 / mpmath.factorial(5)),
            short21(1 / mpmath.factorial(6)), short21(1 / mpmath.factorial(7))]


def fx(v):
    return int(mpmath.nint(v * mpmath.power(2, FX)))


def limbs(i):
    return [(i >> (64 * k)) & ((1 << 64) - 1) for k in range(3)]  # little-endian limbs


def ln2_fx():
    return fx(mpmath.log(2))


def invfact_fx():
    return [fx(1 / mpmath.factorial(i)) for i in range(18)]


def main():
    h, m, l = ln2n_split()
    print(f"#define NKX_INVLN2N {invln2n().hex()}")
    for i, c in enumerate(coeffs()):
        print(f"#define NKX_C{i + 3} {c.hex()}")
    print(f"#define NKX_L2N_H {h.hex()}\n#define NKX_L2N_M {m.hex()}\n#define NKX_L2N_L {l.hex()}")
    print("/* 2^(j/128) = hi + lo */")
    for j, (a, b) in enumerate(table()):
        print(f"    {{{a.hex()}, {b.hex()}}},  /* {j} */")
    print("/* ln2 * 2^190 */")
    print("    " + ", ".join(f"0x{w:016x}ULL" for w in limbs(ln2_fx())))
    print("/* 2^190 / i! */")
    for i, v in enumerate(invfact_fx()):
        print("    {" + ", ".join(f"0x{w:016x}ULL" for w in limbs(v)) + f"}},  /* 1/{i}! */")


if __name__ == "__main__":
    main()
