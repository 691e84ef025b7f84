// nk_exp_dev.hpp -- the correctly rounded exp (nk_exp.h) instantiated for device code.  nk_exp.h is
// the same source the CPU oracle compiles, so every Bratu residual / JVP / FD value is bit-identical
// to the oracle's (bratu.jl:21's lam * exp(u)).
//
// Device forms: every lane runs the branch-free fast phase (nkx_exp_fast; the stencils pass the table
// as an LDS copy).  The lanes it does not settle -- about 2^-18 of inputs, plus non-finite / out-of-range
// ones -- take the exact phase either
//   nk_exp_lane  per lane, divergently, in vector registers: the stencil marches (k_st2d), allocated so
//                this cold code's registers never displace the hot loop's, or
//   nk_exp_t     one lane at a time for the whole wave: the lane's x read into scalar registers
//                (readlane), the exact phase run as wave-uniform scalar code (k_exp, batched JVPs, 1D).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#define NKX_FN __device__ __forceinline__
#define NKX_SLOW_FN __device__ __forceinline__
#define NKX_CONST static __device__ const
#define NKX_OWN_EXP_T 1
#define NKX_NOUNROLL _Pragma("unroll 1")
#include "nk_exp.h"

// correctly rounded exp(x); `tab` = NKX_T as 256 doubles (an LDS copy in the stencils)
__device__ __forceinline__ double nk_exp_t(double x, const double* tab) {
    double y;
    const int ok = nkx_exp_fast(x, tab, &y);
    unsigned long long rare = __ballot(!ok);
    while (rare) {  // wave-uniform
        const int l = __ffsll(rare) - 1;
        const int lo = __builtin_amdgcn_readlane(__double2loint(x), l);
        const int hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
        const double ys = nkx_exp_rare(__hiloint2double(hi, lo));
        if ((int)(threadIdx.x & 63) == l) y = ys;
        rare &= rare - 1;
    }
    return y;
}

// correctly rounded exp(x) per lane: the exact phase runs divergently (vector registers) in the lanes
// that need it -- for code where little else is live (k_st2d's fixup of the points its march marked)
#ifndef NK_EXP_RARE_CALL
#define NK_EXP_RARE_CALL 1
#endif
// the exact phase as a real call: its registers are the callee's; the caller saves what it keeps in
// the clobbered ones around the call -- in the cold block, never in the loop that contains it
__device__ __attribute__((noinline)) double nk_exp_rare_fn(double x) { return nkx_exp_rare(x); }
__device__ __forceinline__ double nk_exp_lane(double x, const double* tab) {
    double y;
    if (__builtin_expect(nkx_exp_fast(x, tab, &y), 1)) return y;
#if NK_EXP_RARE_CALL
    return nk_exp_rare_fn(x);
#else
    return nkx_exp_rare(x);
#endif
}

// correctly rounded exp(x), table from device memory
__device__ __forceinline__ double nk_exp(double x) { return nk_exp_t(x, &NKX_T[0][0]); }
