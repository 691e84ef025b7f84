/* nk_exp.h -- correctly rounded exp(x) for binary64, round-to-nearest-even.
 *
 * ONE source for every exp the Bratu path evaluates, on the device and in the oracle:
 * `bratu!`'s lam * exp(u) (/root/reference/examples/bratu.jl:21) and its Enzyme tangent
 * lam * exp(u) * v (src/Ariadne.jl:48-57).  The HIP stencils (nk_stencil.hpp, nk_batch.hip,
 * nk_resident.hip, the nk_vexp primitive) and the CPU oracle (oracle/nk_oracle.c, test
 * infrastructure) include this file, so both compute bit-identical results; and because the
 * result is the correctly rounded exp, it is the same double any correctly rounded libm returns
 * (Julia's Base.exp, the reference's, is faithful but not proven correctly rounded: the two agree
 * wherever Base.exp rounds correctly, e.g. exp(2.0) == 7.38905609893065 of test/runtests.jl:38).
 *
 * Algorithm (Ziv's strategy, two phases):
 *   fast  x = k ln2/128 + r, |r| <= 1.125 ln2/256 (Cody-Waite, ln2/128 in three parts, r as a
 *         double-double); expm1(r) = r + r^2/2 + r^3 P(r) with r^2 exact (fma) and the
 *         cubic tail in doubles; 2^(j/128) from a 128-entry double-double table; the result
 *         zh + zl carries a relative error below 2^-76 (bound in DESIGN.md; measured max
 *         ~2^-79 over 10^6 inputs, tests/test_exp.py).  A one-fma rounding test (nkx_exp_fast)
 *         shows whether every value within 2^-73 zh of zh + zl rounds to zh; then zh is the
 *         correctly rounded result.
 *   slow  (about 2^-18 of inputs, plus the subnormal and overflow bands): exact fixed-point
 *         arithmetic on 192-bit integers (Q2.190): x converted exactly, r = x - k ln2 with ln2
 *         to 2^-190, exp(r/256) by a 17-term Horner series with 1/i! to 2^-190, eight
 *         squarings, then one rounding to nearest-even straight from the 192-bit value
 *         (normal or subnormal).  Error < 2^-170 relative, far inside the Lefevre-Muller
 *         worst case for binary64 exp (exp(x) never lies closer than ~2^-113 relative to a
 *         rounding boundary for a double x outside the trivial |x| < 2^-54 range).
 *
 * Bit-for-bit identical on gfx950 and x86-64: only IEEE-754 +, -, *, fma (correctly rounded
 * everywhere), rint, ldexp and integer arithmetic; the includer compiles with
 * -ffp-contract=off so the compiler fuses nothing on its own.
 *
 * The includer defines
 *   NKX_FN       qualifiers of the fast path (device: __device__ __forceinline__; C: static inline)
 *   NKX_SLOW_FN  qualifiers of the rare path (device: __device__ __attribute__((noinline)))
 *   NKX_CONST    storage qualifier of the tables (device: static __device__ const; C: static const)
 *   NKX_NOUNROLL (optional) a loop pragma for the exact phase's two long loops (device: unroll 1)
 */
#ifndef NK_EXP_H
#define NK_EXP_H

#ifndef NKX_NOUNROLL
#define NKX_NOUNROLL
#endif

typedef unsigned long long nkx_u64;
typedef unsigned __int128 nkx_u128;

#define NKX_INVLN2N 0x1.7154700000000p+7
#define NKX_L2N_H 0x1.62e4200000000p-8
#define NKX_L2N_M 0x1.fdf473de6af28p-29
#define NKX_L2N_L -0x1.c4c67fc0d0951p-83
/* Taylor coefficients of the cubic tail r^3 (1/6 + r/24 + r^2/120 + r^3/720 + r^4/5040); 1/720 and 1/5040
   to 21 bits, like INVLN2N and L2N_H (gfx950 takes such doubles as 32-bit literals: fewer scalar registers) */
#define NKX_C3 0x1.5555555555555p-3
#define NKX_C4 0x1.5555555555555p-5
#define NKX_C5 0x1.1111111111111p-7
#define NKX_C6 0x1.6c16c00000000p-10
#define NKX_C7 0x1.a01a000000000p-13
#define NKX_INVLN2 0x1.71547652b82fep+0

/* 2^(j/128) = hi + lo */
NKX_CONST double NKX_T[128][2] = {
    {0x1.0000000000000p+0, 0x0.0p+0},  /* 0 */
    {0x1.0163da9fb3335p+0, 0x1.b61299ab8cdb7p-54},  /* 1 */
    {0x1.02c9a3e778061p+0, -0x1.19083535b085dp-56},  /* 2 */
    {0x1.04315e86e7f85p+0, -0x1.0a31c1977c96ep-54},  /* 3 */
    {0x1.059b0d3158574p+0, 0x1.d73e2a475b465p-55},  /* 4 */
    {0x1.0706b29ddf6dep+0, -0x1.c91dfe2b13c27p-55},  /* 5 */
    {0x1.0874518759bc8p+0, 0x1.186be4bb284ffp-57},  /* 6 */
    {0x1.09e3ecac6f383p+0, 0x1.1487818316136p-54},  /* 7 */
    {0x1.0b5586cf9890fp+0, 0x1.8a62e4adc610bp-54},  /* 8 */
    {0x1.0cc922b7247f7p+0, 0x1.01edc16e24f71p-54},  /* 9 */
    {0x1.0e3ec32d3d1a2p+0, 0x1.03a1727c57b53p-59},  /* 10 */
    {0x1.0fb66affed31bp+0, -0x1.b9bedc44ebd7bp-57},  /* 11 */
    {0x1.11301d0125b51p+0, -0x1.6c51039449b3ap-54},  /* 12 */
    {0x1.12abdc06c31ccp+0, -0x1.1b514b36ca5c7p-58},  /* 13 */
    {0x1.1429aaea92de0p+0, -0x1.32fbf9af1369ep-54},  /* 14 */
    {0x1.15a98c8a58e51p+0, 0x1.2406ab9eeab0ap-55},  /* 15 */
    {0x1.172b83c7d517bp+0, -0x1.19041b9d78a76p-55},  /* 16 */
    {0x1.18af9388c8deap+0, -0x1.11023d1970f6cp-54},  /* 17 */
    {0x1.1a35beb6fcb75p+0, 0x1.e5b4c7b4968e4p-55},  /* 18 */
    {0x1.1bbe084045cd4p+0, -0x1.95386352ef607p-54},  /* 19 */
    {0x1.1d4873168b9aap+0, 0x1.e016e00a2643cp-54},  /* 20 */
    {0x1.1ed5022fcd91dp+0, -0x1.1df98027bb78cp-54},  /* 21 */
    {0x1.2063b88628cd6p+0, 0x1.dc775814a8495p-55},  /* 22 */
    {0x1.21f49917ddc96p+0, 0x1.2a97e9494a5eep-55},  /* 23 */
    {0x1.2387a6e756238p+0, 0x1.9b07eb6c70573p-54},  /* 24 */
    {0x1.251ce4fb2a63fp+0, 0x1.ac155bef4f4a4p-55},  /* 25 */
    {0x1.26b4565e27cddp+0, 0x1.2bd339940e9d9p-55},  /* 26 */
    {0x1.284dfe1f56381p+0, -0x1.a4c3a8c3f0d7ep-54},  /* 27 */
    {0x1.29e9df51fdee1p+0, 0x1.612e8afad1255p-55},  /* 28 */
    {0x1.2b87fd0dad990p+0, -0x1.10adcd6381aa4p-59},  /* 29 */
    {0x1.2d285a6e4030bp+0, 0x1.0024754db41d5p-54},  /* 30 */
    {0x1.2ecafa93e2f56p+0, 0x1.1ca0f45d52383p-56},  /* 31 */
    {0x1.306fe0a31b715p+0, 0x1.6f46ad23182e4p-55},  /* 32 */
    {0x1.32170fc4cd831p+0, 0x1.a9ce78e18047cp-55},  /* 33 */
    {0x1.33c08b26416ffp+0, 0x1.32721843659a6p-54},  /* 34 */
    {0x1.356c55f929ff1p+0, -0x1.b5cee5c4e4628p-55},  /* 35 */
    {0x1.371a7373aa9cbp+0, -0x1.63aeabf42eae2p-54},  /* 36 */
    {0x1.38cae6d05d866p+0, -0x1.e958d3c9904bdp-54},  /* 37 */
    {0x1.3a7db34e59ff7p+0, -0x1.5e436d661f5e3p-56},  /* 38 */
    {0x1.3c32dc313a8e5p+0, -0x1.efff8375d29c3p-54},  /* 39 */
    {0x1.3dea64c123422p+0, 0x1.ada0911f09ebcp-55},  /* 40 */
    {0x1.3fa4504ac801cp+0, -0x1.7d023f956f9f3p-54},  /* 41 */
    {0x1.4160a21f72e2ap+0, -0x1.ef3691c309278p-58},  /* 42 */
    {0x1.431f5d950a897p+0, -0x1.1c7dde35f7999p-55},  /* 43 */
    {0x1.44e086061892dp+0, 0x1.89b7a04ef80d0p-59},  /* 44 */
    {0x1.46a41ed1d0057p+0, 0x1.c944bd1648a76p-54},  /* 45 */
    {0x1.486a2b5c13cd0p+0, 0x1.3c1a3b69062f0p-56},  /* 46 */
    {0x1.4a32af0d7d3dep+0, 0x1.9cb62f3d1be56p-54},  /* 47 */
    {0x1.4bfdad5362a27p+0, 0x1.d4397afec42e2p-56},  /* 48 */
    {0x1.4dcb299fddd0dp+0, 0x1.8ecdbbc6a7833p-54},  /* 49 */
    {0x1.4f9b2769d2ca7p+0, -0x1.4b309d25957e3p-54},  /* 50 */
    {0x1.516daa2cf6642p+0, -0x1.f768569bd93efp-55},  /* 51 */
    {0x1.5342b569d4f82p+0, -0x1.07abe1db13cadp-55},  /* 52 */
    {0x1.551a4ca5d920fp+0, -0x1.d689cefede59bp-55},  /* 53 */
    {0x1.56f4736b527dap+0, 0x1.9bb2c011d93adp-54},  /* 54 */
    {0x1.58d12d497c7fdp+0, 0x1.295e15b9a1de8p-55},  /* 55 */
    {0x1.5ab07dd485429p+0, 0x1.6324c054647adp-54},  /* 56 */
    {0x1.5c9268a5946b7p+0, 0x1.c4b1b816986a2p-60},  /* 57 */
    {0x1.5e76f15ad2148p+0, 0x1.ba6f93080e65ep-54},  /* 58 */
    {0x1.605e1b976dc09p+0, -0x1.3e2429b56de47p-54},  /* 59 */
    {0x1.6247eb03a5585p+0, -0x1.383c17e40b497p-54},  /* 60 */
    {0x1.6434634ccc320p+0, -0x1.c483c759d8933p-55},  /* 61 */
    {0x1.6623882552225p+0, -0x1.bb60987591c34p-54},  /* 62 */
    {0x1.68155d44ca973p+0, 0x1.038ae44f73e65p-57},  /* 63 */
    {0x1.6a09e667f3bcdp+0, -0x1.bdd3413b26456p-54},  /* 64 */
    {0x1.6c012750bdabfp+0, -0x1.2895667ff0b0dp-56},  /* 65 */
    {0x1.6dfb23c651a2fp+0, -0x1.bbe3a683c88abp-57},  /* 66 */
    {0x1.6ff7df9519484p+0, -0x1.83c0f25860ef6p-55},  /* 67 */
    {0x1.71f75e8ec5f74p+0, -0x1.16e4786887a99p-55},  /* 68 */
    {0x1.73f9a48a58174p+0, -0x1.0a8d96c65d53cp-54},  /* 69 */
    {0x1.75feb564267c9p+0, -0x1.0245957316dd3p-54},  /* 70 */
    {0x1.780694fde5d3fp+0, 0x1.866b80a02162dp-54},  /* 71 */
    {0x1.7a11473eb0187p+0, -0x1.41577ee04992fp-55},  /* 72 */
    {0x1.7c1ed0130c132p+0, 0x1.f124cd1164dd6p-54},  /* 73 */
    {0x1.7e2f336cf4e62p+0, 0x1.05d02ba15797ep-56},  /* 74 */
    {0x1.80427543e1a12p+0, -0x1.27c86626d972bp-54},  /* 75 */
    {0x1.82589994cce13p+0, -0x1.d4c1dd41532d8p-54},  /* 76 */
    {0x1.8471a4623c7adp+0, -0x1.8d684a341cdfbp-55},  /* 77 */
    {0x1.868d99b4492edp+0, -0x1.fc6f89bd4f6bap-54},  /* 78 */
    {0x1.88ac7d98a6699p+0, 0x1.994c2f37cb53ap-54},  /* 79 */
    {0x1.8ace5422aa0dbp+0, 0x1.6e9f156864b27p-54},  /* 80 */
    {0x1.8cf3216b5448cp+0, -0x1.0d55e32e9e3aap-56},  /* 81 */
    {0x1.8f1ae99157736p+0, 0x1.5cc13a2e3976cp-55},  /* 82 */
    {0x1.9145b0b91ffc6p+0, -0x1.dd6792e582524p-54},  /* 83 */
    {0x1.93737b0cdc5e5p+0, -0x1.75fc781b57ebcp-57},  /* 84 */
    {0x1.95a44cbc8520fp+0, -0x1.64b7c96a5f039p-56},  /* 85 */
    {0x1.97d829fde4e50p+0, -0x1.d185b7c1b85d1p-54},  /* 86 */
    {0x1.9a0f170ca07bap+0, -0x1.173bd91cee632p-54},  /* 87 */
    {0x1.9c49182a3f090p+0, 0x1.c7c46b071f2bep-56},  /* 88 */
    {0x1.9e86319e32323p+0, 0x1.824ca78e64c6ep-56},  /* 89 */
    {0x1.a0c667b5de565p+0, -0x1.359495d1cd533p-54},  /* 90 */
    {0x1.a309bec4a2d33p+0, 0x1.6305c7ddc36abp-54},  /* 91 */
    {0x1.a5503b23e255dp+0, -0x1.d2f6edb8d41e1p-54},  /* 92 */
    {0x1.a799e1330b358p+0, 0x1.bcb7ecac563c7p-54},  /* 93 */
    {0x1.a9e6b5579fdbfp+0, 0x1.0fac90ef7fd31p-54},  /* 94 */
    {0x1.ac36bbfd3f37ap+0, -0x1.f9234cae76cd0p-55},  /* 95 */
    {0x1.ae89f995ad3adp+0, 0x1.7a1cd345dcc81p-54},  /* 96 */
    {0x1.b0e07298db666p+0, -0x1.bdef54c80e425p-54},  /* 97 */
    {0x1.b33a2b84f15fbp+0, -0x1.2805e3084d708p-57},  /* 98 */
    {0x1.b59728de5593ap+0, -0x1.c71dfbbba6de3p-54},  /* 99 */
    {0x1.b7f76f2fb5e47p+0, -0x1.5584f7e54ac3bp-56},  /* 100 */
    {0x1.ba5b030a1064ap+0, -0x1.efcd30e54292ep-54},  /* 101 */
    {0x1.bcc1e904bc1d2p+0, 0x1.23dd07a2d9e84p-55},  /* 102 */
    {0x1.bf2c25bd71e09p+0, -0x1.efdca3f6b9c73p-54},  /* 103 */
    {0x1.c199bdd85529cp+0, 0x1.11065895048ddp-55},  /* 104 */
    {0x1.c40ab5fffd07ap+0, 0x1.b4537e083c60ap-54},  /* 105 */
    {0x1.c67f12e57d14bp+0, 0x1.2884dff483cadp-54},  /* 106 */
    {0x1.c8f6d9406e7b5p+0, 0x1.1acbc48805c44p-56},  /* 107 */
    {0x1.cb720dcef9069p+0, 0x1.503cbd1e949dbp-56},  /* 108 */
    {0x1.cdf0b555dc3fap+0, -0x1.dd83b53829d72p-55},  /* 109 */
    {0x1.d072d4a07897cp+0, -0x1.cbc3743797a9cp-54},  /* 110 */
    {0x1.d2f87080d89f2p+0, -0x1.d487b719d8578p-54},  /* 111 */
    {0x1.d5818dcfba487p+0, 0x1.2ed02d75b3707p-55},  /* 112 */
    {0x1.d80e316c98398p+0, -0x1.11ec18beddfe8p-54},  /* 113 */
    {0x1.da9e603db3285p+0, 0x1.c2300696db532p-54},  /* 114 */
    {0x1.dd321f301b460p+0, 0x1.2da5778f018c3p-54},  /* 115 */
    {0x1.dfc97337b9b5fp+0, -0x1.1a5cd4f184b5cp-54},  /* 116 */
    {0x1.e264614f5a129p+0, -0x1.7b627817a1496p-54},  /* 117 */
    {0x1.e502ee78b3ff6p+0, 0x1.39e8980a9cc8fp-55},  /* 118 */
    {0x1.e7a51fbc74c83p+0, 0x1.2d522ca0c8de2p-54},  /* 119 */
    {0x1.ea4afa2a490dap+0, -0x1.e9c23179c2893p-54},  /* 120 */
    {0x1.ecf482d8e67f1p+0, -0x1.c93f3b411ad8cp-54},  /* 121 */
    {0x1.efa1bee615a27p+0, 0x1.dc7f486a4b6b0p-54},  /* 122 */
    {0x1.f252b376bba97p+0, 0x1.3a1a5bf0d8e43p-54},  /* 123 */
    {0x1.f50765b6e4540p+0, 0x1.9d3e12dd8a18bp-54},  /* 124 */
    {0x1.f7bfdad9cbe14p+0, -0x1.dbb12d006350ap-54},  /* 125 */
    {0x1.fa7c1819e90d8p+0, 0x1.74853f3a5931ep-55},  /* 126 */
    {0x1.fd3c22b8f71f1p+0, 0x1.2eb74966579e7p-57},  /* 127 */
};

/* ln2 * 2^190 and 2^190 / i!, little-endian 64-bit limbs */
NKX_CONST nkx_u64 NKX_LN2_FX[3] = {
    0xd03cd0c99ca62d8bULL, 0xf278ece600fcbdabULL, 0x2c5c85fdf473de6aULL
};
NKX_CONST nkx_u64 NKX_INVFACT_FX[18][3] = {
    {0x0000000000000000ULL, 0x0000000000000000ULL, 0x4000000000000000ULL},  /* 1/0! */
    {0x0000000000000000ULL, 0x0000000000000000ULL, 0x4000000000000000ULL},  /* 1/1! */
    {0x0000000000000000ULL, 0x0000000000000000ULL, 0x2000000000000000ULL},  /* 1/2! */
    {0xaaaaaaaaaaaaaaabULL, 0xaaaaaaaaaaaaaaaaULL, 0x0aaaaaaaaaaaaaaaULL},  /* 1/3! */
    {0xaaaaaaaaaaaaaaabULL, 0xaaaaaaaaaaaaaaaaULL, 0x02aaaaaaaaaaaaaaULL},  /* 1/4! */
    {0x8888888888888889ULL, 0x8888888888888888ULL, 0x0088888888888888ULL},  /* 1/5! */
    {0x16c16c16c16c16c1ULL, 0xc16c16c16c16c16cULL, 0x0016c16c16c16c16ULL},  /* 1/6! */
    {0x0340340340340340ULL, 0x4034034034034034ULL, 0x0003403403403403ULL},  /* 1/7! */
    {0x8068068068068068ULL, 0x6806806806806806ULL, 0x0000680680680680ULL},  /* 1/8! */
    {0xb8ef1d2ab6399c7dULL, 0x99c7d560e4472800ULL, 0x00000b8ef1d2ab63ULL},  /* 1/9! */
    {0x78e4b61ddf05c2d9ULL, 0xf5c72ef016d3ea66ULL, 0x00000127e4fb7789ULL},  /* 1/10! */
    {0xdc71e202b72f11b7ULL, 0x44e38fe747e4b837ULL, 0x0000001ae64567f5ULL},  /* 1/11! */
    {0xfd097d8039ee96cfULL, 0x1b12f6a89b530f59ULL, 0x000000023ddb1dffULL},  /* 1/12! */
    {0x75ed09a766eaf7e9ULL, 0x50da12f9470663a4ULL, 0x000000002c248c27ULL},  /* 1/13! */
    {0xbf47c9d519a311b5ULL, 0x180f93a4175be28bULL, 0x0000000003272e95ULL},  /* 1/14! */
    {0x1dd195fd23d7abd9ULL, 0xce67703e23b0cad6ULL, 0x000000000035cfe7ULL},  /* 1/15! */
    {0x61dd195fd23d7abeULL, 0x7ce67703e23b0cadULL, 0x0000000000035cfeULL},  /* 1/16! */
    {0x32eee35ffd4ee91aULL, 0x8ee0615a94d64c0aULL, 0x00000000000032a5ULL},  /* 1/17! */
};

NKX_FN nkx_u64 nkx_bits(double x) {
    union { double d; nkx_u64 u; } v;
    v.d = x;
    return v.u;
}

NKX_FN double nkx_double(nkx_u64 u) {
    union { double d; nkx_u64 u; } v;
    v.u = u;
    return v.d;
}

/* floor(a * b / 2^190), both Q2.190 with a * b < 4 */
NKX_FN void nkx_mul(nkx_u64 o[3], const nkx_u64 a[3], const nkx_u64 b[3]) {
    nkx_u64 p[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 3; ++i) {
        nkx_u64 carry = 0;
        for (int j = 0; j < 3; ++j) {
            nkx_u128 t = (nkx_u128)a[i] * b[j] + p[i + j] + carry;
            p[i + j] = (nkx_u64)t;
            carry = (nkx_u64)(t >> 64);
        }
        p[i + 3] = carry;
    }
    o[0] = (p[2] >> 62) | (p[3] << 2);
    o[1] = (p[3] >> 62) | (p[4] << 2);
    o[2] = (p[4] >> 62) | (p[5] << 2);
}

/* bit `pos` of a 3-limb value (0 beyond 191) */
NKX_FN nkx_u64 nkx_bit(const nkx_u64 y[3], int pos) {
    return pos >= 192 ? 0 : (y[pos >> 6] >> (pos & 63)) & 1;
}

/* any bit strictly below `pos` */
NKX_FN int nkx_any_below(const nkx_u64 y[3], int pos) {
    if (pos > 192) pos = 192;
    for (int l = 0; l < 3; ++l) {
        int lo = 64 * l;
        if (pos <= lo) break;
        nkx_u64 w = y[l];
        if (pos < lo + 64) w &= (((nkx_u64)1) << (pos - lo)) - 1;
        if (w) return 1;
    }
    return 0;
}

/* round-to-nearest-even of y / 2^sh, sh in [1, 192]; the quotient fits 54 bits */
NKX_FN nkx_u64 nkx_round_shift(const nkx_u64 y[3], int sh) {
    nkx_u64 q = 0;
    if (sh < 192) {
        const int li = sh >> 6, bi = sh & 63;
        q = y[li] >> bi;
        if (bi && li < 2) q |= y[li + 1] << (64 - bi);
    }
    const nkx_u64 rb = nkx_bit(y, sh - 1);
    if (rb && (nkx_any_below(y, sh - 1) || (q & 1))) q += 1;
    return q;
}

/* The accurate phase: exact fixed-point evaluation, one final rounding (normal or subnormal).
   Valid for 2^-54 < |x| < 746. */
NKX_SLOW_FN double nkx_exp_slow(double x) {
    const nkx_u64 bits = nkx_bits(x);
    const int neg = (int)(bits >> 63);
    const int e = (int)((bits >> 52) & 0x7ff);
    const nkx_u64 m = (bits & 0xfffffffffffffULL) | (1ULL << 52);
    /* X = |x| 2^190 = m 2^(e - 1075 + 190), exact in 256 bits (shift in [84, 147]) */
    nkx_u64 X[4] = {0, 0, 0, 0};
    const int shift = e - 885;
    const int q = shift >> 6, s = shift & 63;
    X[q] = m << s;
    if (s) X[q + 1] = m >> (64 - s);
    if (neg) { /* two's complement */
        nkx_u64 c = 1;
        for (int l = 0; l < 4; ++l) {
            nkx_u128 t = (nkx_u128)(~X[l]) + c;
            X[l] = (nkx_u64)t;
            c = (nkx_u64)(t >> 64);
        }
    }
    int kk = (int)rint(x * NKX_INVLN2);
    /* R = X - kk * LN2 (two's complement, 256 bits) */
    const nkx_u64 ak = (nkx_u64)(kk < 0 ? -kk : kk);
    nkx_u64 A[4];
    {
        nkx_u64 c = 0;
        for (int l = 0; l < 3; ++l) {
            nkx_u128 t = (nkx_u128)NKX_LN2_FX[l] * ak + c;
            A[l] = (nkx_u64)t;
            c = (nkx_u64)(t >> 64);
        }
        A[3] = c;
    }
    nkx_u64 R[4];
    {
        nkx_u64 c = 0;
        for (int l = 0; l < 4; ++l) {
            /* kk >= 0: R = X - A; kk < 0: R = X + A */
            nkx_u128 t;
            if (kk >= 0) {
                t = (nkx_u128)X[l] - A[l] - c;
                c = (nkx_u64)(t >> 64) ? 1 : 0;
            } else {
                t = (nkx_u128)X[l] + A[l] + c;
                c = (nkx_u64)(t >> 64);
            }
            R[l] = (nkx_u64)t;
        }
    }
    if (R[3] >> 63) { /* r < 0: one ln2 more */
        kk -= 1;
        nkx_u64 c = 0;
        for (int l = 0; l < 4; ++l) {
            nkx_u128 t = (nkx_u128)R[l] + (l < 3 ? NKX_LN2_FX[l] : 0) + c;
            R[l] = (nkx_u64)t;
            c = (nkx_u64)(t >> 64);
        }
    }
    /* r' = r / 256 (0 <= r <= ln2 + tiny, so R[3] == 0) */
    nkx_u64 rr[3];
    rr[0] = (R[0] >> 8) | (R[1] << 56);
    rr[1] = (R[1] >> 8) | (R[2] << 56);
    rr[2] = (R[2] >> 8) | (R[3] << 56);
    /* exp(r') = sum_{i <= 17} r'^i / i!  (Horner) */
    nkx_u64 y[3] = {NKX_INVFACT_FX[17][0], NKX_INVFACT_FX[17][1], NKX_INVFACT_FX[17][2]};
    NKX_NOUNROLL
    for (int i = 16; i >= 0; --i) {
        nkx_u64 t[3];
        nkx_mul(t, y, rr);
        nkx_u64 c = 0;
        for (int l = 0; l < 3; ++l) {
            nkx_u128 s2 = (nkx_u128)t[l] + NKX_INVFACT_FX[i][l] + c;
            y[l] = (nkx_u64)s2;
            c = (nkx_u64)(s2 >> 64);
        }
    }
    NKX_NOUNROLL
    for (int i = 0; i < 8; ++i) { /* exp(r) = exp(r')^256 */
        nkx_u64 t[3];
        nkx_mul(t, y, y);
        y[0] = t[0];
        y[1] = t[1];
        y[2] = t[2];
    }
    /* y in [1, 2 + tiny) as Q2.190: top bit at 190 or 191 */
    const int top = (y[2] >> 63) ? 191 : 190;
    int E = kk + (top - 190); /* exp(x) = 1.f 2^E */
    if (E > 1023) return nkx_double(0x7ff0000000000000ULL);
    if (E >= -1022) {
        nkx_u64 qq = nkx_round_shift(y, top - 52);
        if (qq >> 53) {
            qq >>= 1;
            E += 1;
            if (E > 1023) return nkx_double(0x7ff0000000000000ULL);
        }
        return nkx_double(((nkx_u64)(E + 1023) << 52) | (qq & 0xfffffffffffffULL));
    }
    const int sh = top - 52 + (-1022 - E);
    if (sh > 192) return 0.0;
    return nkx_double(nkx_round_shift(y, sh)); /* a subnormal (or the least normal after carry) */
}

/* The fast phase alone: exp(x) = (zh + zl) 2^m with |zh + zl - exp(x)/2^m| < 2^-76 zh.
   Valid for -708.3 < x < 709.78 and |x| > 2^-54.  `tab` = NKX_T as 256 doubles (hi, lo interleaved):
   the stencils pass a copy in LDS (a table load from global memory would share the in-order vmcnt
   counter with the rows the march keeps in flight, and waiting for it would drain them). */
NKX_FN double nkx_exp_dd(double x, const double* tab, double* zl_out, int* m_out) {
    const double kd = rint(x * NKX_INVLN2N);
    const int k = (int)kd;
    const double rh = fma(kd, -NKX_L2N_H, x); /* exact: kd * H has <= 39 bits, Sterbenz */
    const double ph = kd * NKX_L2N_M;
    const double pl = fma(kd, NKX_L2N_M, -ph);
    const double r1 = rh - ph; /* TwoSum(rh, -ph) */
    const double bb = r1 - rh;
    const double e1 = (rh - (r1 - bb)) + (-ph - bb);
    const double rl = fma(-kd, NKX_L2N_L, e1 - pl); /* r = r1 + rl to ~2^-114 absolute */
    const double sh = r1 * r1;
    const double sl = fma(r1, r1, -sh);
    const double tail = (sh * r1) * fma(r1, fma(r1, fma(r1, fma(r1, NKX_C7, NKX_C6), NKX_C5), NKX_C4), NKX_C3);
    const double h2 = sh * 0.5;
    const double qh = h2 + tail; /* FastTwoSum(h2, tail): |tail| < |h2| */
    const double ql = tail - (qh - h2);
    const double eh = r1 + qh; /* FastTwoSum(r1, qh): |qh| < |r1| */
    const double t = qh - (eh - r1);
    const double el = t + (ql + (rl + fma(sl, 0.5, r1 * rl))); /* expm1(r) = eh + el */
    const int j = k & 127;
    *m_out = (k - j) / 128;
    const double Th = tab[2 * j], Tl = tab[2 * j + 1];
    const double p_h = Th * eh;
    const double p_l = fma(Th, eh, -p_h);
    const double yh = Th + p_h; /* FastTwoSum(Th, p_h) */
    const double y1 = p_h - (yh - Th);
    const double yl = y1 + (p_l + fma(Th, el, fma(Tl, eh, Tl)));
    const double zh = yh + yl; /* FastTwoSum(yh, yl) */
    *zl_out = yl - (zh - yh);
    return zh;
}

/* Everything the fast phase does not settle: NaN, +-inf, overflow, underflow and subnormal results,
   |x| <= 2^-54, and the inputs the Ziv test hands over. */
NKX_SLOW_FN double nkx_exp_rare(double x) {
    if (x != x) return x + x;
    if (!(fabs(x) > 0x1p-54)) return 1.0; /* |x| <= 2^-54 rounds to 1 */
    if (x > 709.79) return nkx_double(0x7ff0000000000000ULL);
    if (x < -745.14) return 0.0;
    return nkx_exp_slow(x);
}

/* The fast phase with its rounding test: returns 1 and *y = exp(x) correctly rounded when it settles x,
   else 0 (then nkx_exp_rare(x) does).  Branch-free: the fast phase runs on x clamped into its range
   (every conversion stays defined) and one combined condition decides.  The Ziv test (CRlibm's form):
   zh = RN(zh + zl) already; if also RN(zh + zl (1 + 2^-18)) == zh (one fma), every value within
   eps zh of zh + zl rounds to zh for any eps < 2^-73 -- the rounding boundary on zl's side sits
   ulp_b / 2 from zh with ulp_b >= 2^-53 zh (the smaller ulp below a power of two included): where
   |zl| >= ulp_b / 4 the test leaves a margin 2^-18 |zl| >= 2^-73 zh, elsewhere the boundary is more
   than ulp_b / 4 >= 2^-55 zh away.  The fast phase's bound is eps = 2^-76 (measured 2^-79.2).  The
   test fails for about 2^-18 of inputs, and for NaN. */
NKX_FN int nkx_exp_fast(double x, const double* tab, double* y) {
    const double xc = fmin(fmax(x, -708.3), 709.78); /* == x inside the fast range */
    double zl;
    int m;
    const double zh = nkx_exp_dd(xc, tab, &zl, &m);
    *y = ldexp(zh, m);
    return (fma(zl, 0x1.00004p0, zh) == zh) & (x < 709.78) & (x > -708.3);
}

#ifndef NKX_OWN_EXP_T /* (the device header defines its own: one wave-uniform pass over the rare lanes) */
/* correctly rounded exp(x); `tab` as for nkx_exp_dd */
NKX_FN double nk_exp_t(double x, const double* tab) {
    double y;
    if (nkx_exp_fast(x, tab, &y)) return y;
    return nkx_exp_rare(x);
}

/* correctly rounded exp(x), table from NKX_T */
NKX_FN double nk_exp(double x) { return nk_exp_t(x, &NKX_T[0][0]); }
#endif

#endif /* NK_EXP_H */
