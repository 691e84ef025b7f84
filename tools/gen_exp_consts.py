"""Generate the constants of the correctly rounded exp (newtonkrylov.jl_amd/csrc/nk_exp.h) with mpmath.

Prints C initialisers (hex-float doubles and 64-bit limbs); nk_exp.h holds their output verbatim, and
tests/test_exp.py re-derives every constant from this script's functions and compares.

  NKX_T[j] = (hi, lo)  2^(j/128) = hi + lo to ~107 bits, j = 0..127 (the fast path's table)
  L2N_H/M/L            ln2/128 = H + M + L, H with 33 significant bits (kd * H exact for |kd| < 2^20)
  INVLN2N              128/ln2 rounded
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
    hi = mpmath.ldexp(mpmath.floor(mpmath.ldexp(m, 33)), e - 33)  # 33 significant bits
    h = float(hi)
    assert mpmath.mpf(h) == hi
    mid = dbl(c - hi)
    low = dbl(c - hi - mpmath.mpf(mid))
    return h, mid, low


def invln2n():
    return dbl(N / mpmath.log(2))


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
