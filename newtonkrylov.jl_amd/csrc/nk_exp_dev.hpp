// nk_exp_dev.hpp -- the correctly rounded exp (nk_exp.h) instantiated for device code.  nk_exp.h is
// the same source the CPU oracle compiles, so every Bratu residual / JVP / FD value is bit-identical
// to the oracle's (bratu.jl:21's lam * exp(u)).  The fast phase inlines into the stencils; the rare
// exact phase (~2^-18 of inputs, plus the subnormal / overflow bands) is one call.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#define NKX_FN __device__ __forceinline__
#ifndef NKX_SLOW_FN
#define NKX_SLOW_FN __device__ __attribute__((noinline))
#endif
#define NKX_CONST static __device__ const
#include "nk_exp.h"
