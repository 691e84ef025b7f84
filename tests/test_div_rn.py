"""div_rn (csrc/nk_stencil.hpp): the stencils' exact quotient RN(a / b) from a precomputed RN(1 / b) --
Markstein's correction, three fma-class operations in place of the division sequence.  Checked here on the
CPU (gcc, the same operations and guard compiled from a C copy of the five lines) against IEEE division on
2.2e8 quotients: the stencils' divisors (h^2 of the grid sizes the tests and bench use, FD steps eps,
normalisation scales h) and random ones, dividends over 2^-60 .. 2^60 of both signs, half of them one ulp
below a random double.  The device form is pinned by the bitwise GPU parity tests (tests/test_hip*.py)."""
import os
import subprocess
import tempfile

SRC = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
static uint64_t s = 88172645463325252ULL;
static uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double rnd(double lo, double hi) { return lo + (hi - lo) * ((xr() >> 11) * 0x1.0p-53); }
static double div_rn(double a, double b, double yb) {   /* nk_stencil.hpp's div_rn */
    const double q0 = a * yb;
    const double r = fma(-q0, b, a);
    const double q1 = fma(r, yb, q0);
    const double aa = fabs(a), aq = fabs(q0);
    if (aa >= 0x1p-900 && aq >= 0x1p-900 && aq <= 0x1p1000) return q1;
    return a / b;
}
int main(void) {
    long bad = 0, tot = 0;
    double bs[64];
    int nb = 0;
    const int ns[] = {64, 100, 127, 500, 1000, 2048, 4095, 4096, 8192, 16384, 3, 7};
    for (int i = 0; i < 12; ++i) { const double h = 1.0 / (ns[i] + 1); bs[nb++] = h * h; }
    for (int i = 0; i < 20; ++i) bs[nb++] = rnd(1e-9, 1e-7);
    for (int i = 0; i < 20; ++i) bs[nb++] = ldexp(rnd(1.0, 2.0), (int)(xr() % 200) - 100);
    bs[nb++] = nextafter(2.0, 0.0); bs[nb++] = 1.0 + 0x1p-52; bs[nb++] = 3.0;
    for (int ib = 0; ib < nb; ++ib) {
        const double b = bs[ib], y = 1.0 / b;
        for (long k = 0; k < 4000000; ++k) {
            double a = ldexp(rnd(1.0, 2.0), (int)(xr() % 120) - 60) * ((xr() & 1) ? 1 : -1);
            if (k & 1) a = nextafter(a, 0.0);
            ++tot;
            if (div_rn(a, b, y) != a / b) ++bad;
        }
        if (div_rn(0.0, b, y) != 0.0 / b || signbit(div_rn(-0.0, b, y)) != signbit(-0.0 / b)) ++bad;
    }
    printf("%ld %ld\n", bad, tot);
    return 0;
}
"""


def test_div_rn_matches_ieee_division():
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "t.c"), os.path.join(d, "t")
        with open(c, "w") as f:
            f.write(SRC)
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe, c, "-lm"], check=True)
        bad, tot = map(int, subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split())
    assert tot == 220_000_000 and bad == 0
