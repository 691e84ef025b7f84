// nk_kernels.hip -- the hand-written gfx950 kernels of the JFNK inner loop and their launchers.
//
// Every kernel here is HBM-bound (fp64, ~1 flop/B): no MFMA.  Design rules applied:
//  * 256-thread blocks (4 waves of 64), 16-B (double2) loads/stores wherever the row length is
//    even, grid-stride streaming for BLAS-1 with a fixed grid so reductions are deterministic.
//  * Stencils march along the slowest axis keeping three planes of the stencil field in
//    registers (one HBM read per input per point); x-neighbours come from the neighbouring
//    lane by cross-lane shuffle, only the two wave-edge lanes load their outer column.
//  * XCD-aware tile order: the 8 XCDs each take a contiguous band of tiles, so the halo rows
//    two vertically adjacent tiles share are read on the same XCD.
//  * Reductions never use atomics: each block writes one partial; the NEXT kernel (or the
//    finaliser) sums the partials in a fixed order -- run-to-run bit reproducible.
//  * -ffp-contract=off: stencil expressions round exactly as the reference writes them
//    (((p - 2c) + m) / (h*h), bratu.jl:19, heat_2D.jl:65).  axpy-type updates use fma()
//    explicitly (the oracle uses the same convention), so elementwise results are bit-identical
//    to the CPU oracle; only exp (ocml vs glibc, <= 1 ulp) and reduction order differ.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "nk_stencil.hpp"

namespace nk {
namespace {

// ------------------------------------------------------------------------------ BLAS-1
// Block-contiguous chunks of `len` elements (a multiple of the block size), threads interleaved
// inside the chunk: each block streams one address range -- fewer DRAM page switches than the
// grid-stride order once the vectors outgrow the Infinity Cache (tools/stream_probe.py).
struct Chunk {
    int64_t lo, hi;
};
__device__ __forceinline__ Chunk block_chunk(int64_t len) {
    const int64_t per = ((len + gridDim.x - 1) / gridDim.x + kBlock - 1) / kBlock * kBlock;
    const int64_t lo = (int64_t)blockIdx.x * per;
    return Chunk{lo, lo + per < len ? lo + per : len};
}
#define NK_CHUNKED(i, len)                    \
    const Chunk ck_ = block_chunk(len);       \
    for (int64_t i = ck_.lo + threadIdx.x; i < ck_.hi; i += kBlock)
#define NK_GRID_STRIDE2(i) NK_CHUNKED(i, n >> 1)
#define NK_TAIL (((n & 1) != 0) && blockIdx.x == 0 && threadIdx.x == 0)

__global__ __launch_bounds__(kBlock) void k_dot(int64_t n, const double* __restrict__ x, const double* __restrict__ y,
                                               double* __restrict__ part, int fin) {
    __shared__ double sh[kShN];
    const double2* x2 = reinterpret_cast<const double2*>(x);
    const double2* y2 = reinterpret_cast<const double2*>(y);
    double acc = 0.0;
    NK_GRID_STRIDE2(i) {
        const double2 a = x2[i], b = y2[i];
        acc = fma(a.x, b.x, acc);
        acc = fma(a.y, b.y, acc);
    }
    if (NK_TAIL) acc = fma(x[n - 1], y[n - 1], acc);
    publish(acc, part, fin, sh);
}

__global__ __launch_bounds__(kBlock) void k_sumsq(int64_t n, const double* __restrict__ x, double* __restrict__ part, int fin) {
    __shared__ double sh[kShN];
    const double2* x2 = reinterpret_cast<const double2*>(x);
    double acc = 0.0;
    NK_GRID_STRIDE2(i) {
        const double2 a = x2[i];
        acc = fma(a.x, a.x, acc);
        acc = fma(a.y, a.y, acc);
    }
    if (NK_TAIL) acc = fma(x[n - 1], x[n - 1], acc);
    publish(acc, part, fin, sh);
}

// dst[0] = Σ in (or its sqrt); `mirror` (optional): the same value into mapped host memory, so
// the host can read it after the stream event without a separate device-to-host copy
__global__ __launch_bounds__(kBlock) void k_finalize(const double* __restrict__ in, int len, double* __restrict__ dst, int sqrt_it,
                                                    double* __restrict__ mirror) {
    __shared__ double sh[kShN];
    const double t = reduce_input(in, len, sh);
    if (threadIdx.x == 0) {
        const double r = sqrt_it ? sqrt(t) : t;
        dst[0] = r;
        if (mirror) mirror[0] = r;
    }
}

__global__ __launch_bounds__(kBlock) void k_axpy(int64_t n, double s, const double* __restrict__ x, double* __restrict__ y) {
    const double2* x2 = reinterpret_cast<const double2*>(x);
    double2* y2 = reinterpret_cast<double2*>(y);
    NK_GRID_STRIDE2(i) {
        const double2 a = x2[i];
        double2 b = y2[i];
        b.x = fma(s, a.x, b.x);
        b.y = fma(s, a.y, b.y);
        y2[i] = b;
    }
    if (NK_TAIL) y[n - 1] = fma(s, x[n - 1], y[n - 1]);
}

// y = s x + y with the partials of ||y||^2 (the Newton update and the next FD step's ||u||)
__global__ __launch_bounds__(kBlock) void k_axpy_sumsq(int64_t n, double s, const double* __restrict__ x,
                                                      double* __restrict__ y, double* __restrict__ part, int fin) {
    __shared__ double sh[kShN];
    const double2* x2 = reinterpret_cast<const double2*>(x);
    double2* y2 = reinterpret_cast<double2*>(y);
    double acc = 0.0;
    NK_GRID_STRIDE2(i) {
        const double2 a = x2[i];
        double2 b = y2[i];
        b.x = fma(s, a.x, b.x);
        b.y = fma(s, a.y, b.y);
        y2[i] = b;
        acc = fma(b.x, b.x, acc);
        acc = fma(b.y, b.y, acc);
    }
    if (NK_TAIL) {
        const double b = fma(s, x[n - 1], y[n - 1]);
        y[n - 1] = b;
        acc = fma(b, b, acc);
    }
    publish(acc, part, fin, sh);
}

__global__ __launch_bounds__(kBlock) void k_axpby(int64_t n, double s, const double* __restrict__ x, double t,
                                                 double* __restrict__ y) {
    const double2* x2 = reinterpret_cast<const double2*>(x);
    double2* y2 = reinterpret_cast<double2*>(y);
    NK_GRID_STRIDE2(i) {
        const double2 a = x2[i];
        double2 b = y2[i];
        b.x = fma(t, b.x, s * a.x);
        b.y = fma(t, b.y, s * a.y);
        y2[i] = b;
    }
    if (NK_TAIL) y[n - 1] = fma(t, y[n - 1], s * x[n - 1]);
}

__global__ __launch_bounds__(kBlock) void k_scal(int64_t n, double s, double* __restrict__ x) {
    double2* x2 = reinterpret_cast<double2*>(x);
    NK_GRID_STRIDE2(i) {
        double2 a = x2[i];
        a.x = s * a.x;
        a.y = s * a.y;
        x2[i] = a;
    }
    if (NK_TAIL) x[n - 1] = s * x[n - 1];
}

__global__ __launch_bounds__(kBlock) void k_copy(int64_t n, double* __restrict__ y, const double* __restrict__ x) {
    const double2* x2 = reinterpret_cast<const double2*>(x);
    double2* y2 = reinterpret_cast<double2*>(y);
    NK_GRID_STRIDE2(i) { y2[i] = x2[i]; }
    if (NK_TAIL) y[n - 1] = x[n - 1];
}

__global__ __launch_bounds__(kBlock) void k_fill(int64_t n, double* __restrict__ x, double v) {
    double2* x2 = reinterpret_cast<double2*>(x);
    NK_GRID_STRIDE2(i) { x2[i] = make_double2(v, v); }
    if (NK_TAIL) x[n - 1] = v;
}

__global__ __launch_bounds__(kBlock) void k_divcopy(int64_t n, double* __restrict__ y, const double* __restrict__ x, double s) {
    const double2* x2 = reinterpret_cast<const double2*>(x);
    double2* y2 = reinterpret_cast<double2*>(y);
    NK_GRID_STRIDE2(i) {
        const double2 a = x2[i];
        y2[i] = make_double2(a.x / s, a.y / s);
    }
    if (NK_TAIL) y[n - 1] = x[n - 1] / s;
}

// y = exp.(x) with the stencils' correctly rounded exp (nk_exp.h): the primitive a user residual calls
// for its transcendental, so it evaluates exactly what the oracle does (no alignment assumed: any views)
__global__ __launch_bounds__(kBlock) void k_exp(int64_t n, double* __restrict__ y, const double* __restrict__ x) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) y[i] = nk_exp(x[i]);
}

__global__ __launch_bounds__(kBlock) void k_ref(int64_t n, double* __restrict__ x, double* __restrict__ y, double c, double s) {
    double2* x2 = reinterpret_cast<double2*>(x);
    double2* y2 = reinterpret_cast<double2*>(y);
    NK_GRID_STRIDE2(i) {
        const double2 a = x2[i], b = y2[i];
        x2[i] = make_double2(c * a.x + s * b.x, c * a.y + s * b.y);
        y2[i] = make_double2(s * a.x - c * b.x, s * a.y - c * b.y);
    }
    if (NK_TAIL) {
        const double a = x[n - 1], b = y[n - 1];
        x[n - 1] = c * a + s * b;
        y[n - 1] = s * a - c * b;
    }
}

// One fused MGS pass (Krylov.jl gmres! inner loop):
//   h = <V_i, q>   (reduced from the previous kernel's partials, fixed order)
//   q = q - h V_i  (kaxpy!(n, -h, V_i, q) == fma(-h, V_i, q))
//   partials of <V_{i+1}, q>  (or <q, q> on the last pass: h_{k+1,k} = ||q||)
// 32 B/point (24 on the last pass) instead of the 40 B of separate kdot + kaxpy!.
// U independent 16-B loads per stream are issued before any use (memory-level parallelism);
// NT marks the loads/stores non-temporal (streams that are not re-read soon).

template <bool NT>
__device__ __forceinline__ dx2 ld2(const dx2* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NT>
__device__ __forceinline__ void st2(dx2* p, dx2 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// rev = 1 sweeps the vectors from the end: consecutive passes alternate direction so each pass
// starts on the lines the previous pass touched last (still in the 256 MB Infinity Cache).
// CH = true: block-contiguous chunks (each block sweeps its own range, threads interleaved) instead
// of the grid-stride order -- fewer DRAM page switches once the vectors outgrow the Infinity Cache.
template <bool HAS_NEXT, int U, bool NT, bool NTW = false, bool CH = false, bool NTQ = false>
__global__ __launch_bounds__(kBlock) void k_mgs_pass(int64_t n, double* __restrict__ q, const double* __restrict__ vi,
                                                    const double* __restrict__ vnext, const double* __restrict__ red_in,
                                                    int red_len, double* __restrict__ h_out, double* __restrict__ h_host,
                                                    double* __restrict__ part,
                                                    int rev, int fin) {
    __shared__ double sh[kShN];
    dx2* q2 = reinterpret_cast<dx2*>(q);
    const dx2* v2 = reinterpret_cast<const dx2*>(vi);
    const dx2* w2 = reinterpret_cast<const dx2*>(vnext);
    const int64_t n2 = n >> 1;
    int64_t i0, st, lim;
    if constexpr (CH) {
        const int64_t per = ((n2 + gridDim.x - 1) / gridDim.x + kBlock - 1) / kBlock * kBlock;
        i0 = (int64_t)blockIdx.x * per + threadIdx.x;
        lim = (int64_t)(blockIdx.x + 1) * per < n2 ? (int64_t)(blockIdx.x + 1) * per : n2;
        st = kBlock;
    } else {
        i0 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
        lim = n2;
        st = (int64_t)gridDim.x * kBlock;
    }
    const int64_t base = rev ? n2 - 1 : 0, sgn = rev ? -1 : 1;
    int64_t i = i0;
    // prologue: the first U stream loads go out before the partial-sum reduction, so h's L2 round
    // trip overlaps with HBM latency instead of preceding it
    dx2 a[U], bv[U], cv[U];
    bool have = i + (U - 1) * st < lim;
    if (have) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t e = base + sgn * (i + u * st);
            a[u] = ld2<NTQ>(q2 + e);
            bv[u] = ld2<NT>(v2 + e);
            if constexpr (HAS_NEXT) cv[u] = ld2<NTW>(w2 + e);
        }
    }
    const double h = reduce_input(red_in, red_len, sh);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *h_out = h;
        if (h_host) *h_host = h;  // mapped host mirror of the Hessenberg column
    }
    const double mh = -h;
    double acc = 0.0;
    for (; have; i += U * st, have = i + (U - 1) * st < lim) {
        if (i != i0) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t e = base + sgn * (i + u * st);
                a[u] = ld2<NTQ>(q2 + e);
                bv[u] = ld2<NT>(v2 + e);
                if constexpr (HAS_NEXT) cv[u] = ld2<NTW>(w2 + e);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            a[u].x = fma(mh, bv[u].x, a[u].x);
            a[u].y = fma(mh, bv[u].y, a[u].y);
            st2<NTQ>(q2 + base + sgn * (i + u * st), a[u]);
            if constexpr (HAS_NEXT) {
                acc = fma(cv[u].x, a[u].x, acc);
                acc = fma(cv[u].y, a[u].y, acc);
            } else {
                acc = fma(a[u].x, a[u].x, acc);
                acc = fma(a[u].y, a[u].y, acc);
            }
        }
    }
    for (; i < lim; i += st) {
        const int64_t e = base + sgn * i;
        dx2 a = q2[e];
        const dx2 b = ld2<NT>(v2 + e);
        a.x = fma(mh, b.x, a.x);
        a.y = fma(mh, b.y, a.y);
        q2[e] = a;
        if constexpr (HAS_NEXT) {
            const dx2 c = ld2<NTW>(w2 + e);
            acc = fma(c.x, a.x, acc);
            acc = fma(c.y, a.y, acc);
        } else {
            acc = fma(a.x, a.x, acc);
            acc = fma(a.y, a.y, acc);
        }
    }
    if (NK_TAIL) {
        const double a = fma(mh, vi[n - 1], q[n - 1]);
        q[n - 1] = a;
        acc = HAS_NEXT ? fma(vnext[n - 1], a, acc) : fma(a, a, acc);
    }
    publish(acc, part, fin, sh);
}

struct UpdArgs {
    const double* V[kMaxUpdateVecs];
    double* x;
    double* u;           // Newton update fused in: u -= x_final (x itself is not stored), partials of ||u||^2
    double* xr;
    const double* y;
    double* part;
    int64_t n;
    int k, first, last, restart, fin;
};

// xr = Σ y_i V_i (the kaxpy! chain of gmres!, from xr = 0); on the last chunk x = x + xr
// (restart) or x = xr; optional partials of ||x||^2.  16-B accesses; V loads non-temporal.
// U elements (16 B each) per thread and iteration, all their loads issued before any store: with
// the few streams of a short solve (k = 1..3 in the heat time steps) one element per thread leaves
// too few bytes in flight per CU.
template <int U>
__device__ __forceinline__ void update_elems(const UpdArgs& A, const double* yv, int64_t i, double& acc) {
    dx2 t[U];
#pragma unroll
    for (int e = 0; e < U; ++e) t[e] = A.first ? dx2{0.0, 0.0} : reinterpret_cast<const dx2*>(A.xr)[i + e * kBlock];
    dx2 x0[U], uv[U];
    if (A.last) {
#pragma unroll
        for (int e = 0; e < U; ++e) {
            if (A.restart) x0[e] = reinterpret_cast<const dx2*>(A.x)[i + e * kBlock];
            if (A.u) uv[e] = reinterpret_cast<const dx2*>(A.u)[i + e * kBlock];
        }
    }
#pragma unroll
    for (int m = 0; m < kMaxUpdateVecs; ++m)  // compile-time indices keep yv in registers
        if (m < A.k) {
            dx2 v[U];
#pragma unroll
            for (int e = 0; e < U; ++e) v[e] = __builtin_nontemporal_load(reinterpret_cast<const dx2*>(A.V[m]) + i + e * kBlock);
#pragma unroll
            for (int e = 0; e < U; ++e) {
                t[e].x = fma(yv[m], v[e].x, t[e].x);
                t[e].y = fma(yv[m], v[e].y, t[e].y);
            }
        }
#pragma unroll
    for (int e = 0; e < U; ++e) {
        if (A.last) {
            dx2 xv = t[e];
            if (A.restart) {
                xv.x = fma(1.0, t[e].x, x0[e].x);
                xv.y = fma(1.0, t[e].y, x0[e].y);
            }
            if (A.u) {  // u .-= 1 .* d, exactly kaxpy!(n, -1, x, u) on the x that would have been stored
                uv[e].x = fma(-1.0, xv.x, uv[e].x);
                uv[e].y = fma(-1.0, xv.y, uv[e].y);
                reinterpret_cast<dx2*>(A.u)[i + e * kBlock] = uv[e];
                xv = uv[e];  // the norm below is ||u||
            } else {
                reinterpret_cast<dx2*>(A.x)[i + e * kBlock] = xv;
            }
            acc = fma(xv.x, xv.x, acc);
            acc = fma(xv.y, xv.y, acc);
        } else {
            reinterpret_cast<dx2*>(A.xr)[i + e * kBlock] = t[e];
        }
    }
}

template <int U>
__global__ __launch_bounds__(kBlock) void k_update_x(UpdArgs A) {
    __shared__ double sh[kShN];
    const int64_t n = A.n;
    double yv[kMaxUpdateVecs];
#pragma unroll
    for (int m = 0; m < kMaxUpdateVecs; ++m) yv[m] = m < A.k ? A.y[m] : 0.0;
    double acc = 0.0;
    const Chunk ck = block_chunk(n >> 1);
    int64_t i = ck.lo + threadIdx.x;
    for (; i + (U - 1) * kBlock < ck.hi; i += U * kBlock) update_elems<U>(A, yv, i, acc);
    for (; i < ck.hi; i += kBlock) update_elems<1>(A, yv, i, acc);
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
        const int64_t i = n - 1;
        double t = A.first ? 0.0 : A.xr[i];
#pragma unroll
        for (int m = 0; m < kMaxUpdateVecs; ++m)
            if (m < A.k) t = fma(yv[m], A.V[m][i], t);
        if (A.last) {
            double xv = A.restart ? fma(1.0, t, A.x[i]) : t;
            if (A.u) {
                xv = fma(-1.0, xv, A.u[i]);
                A.u[i] = xv;
            } else {
                A.x[i] = xv;
            }
            acc = fma(xv, xv, acc);
        } else {
            A.xr[i] = t;
        }
    }
    if (A.part) publish(acc, A.part, A.fin, sh);
}

__global__ __launch_bounds__(kBlock) void k_cg_update(int64_t n, double alpha, double* __restrict__ x, double* __restrict__ r,
                                                     const double* __restrict__ p, const double* __restrict__ Ap,
                                                     double* __restrict__ part, int fin) {
    __shared__ double sh[kShN];
    double acc = 0.0;
    const double ma = -alpha;
    NK_CHUNKED(i, n) {
        x[i] = fma(alpha, p[i], x[i]);
        const double rv = fma(ma, Ap[i], r[i]);
        r[i] = rv;
        acc = fma(rv, rv, acc);
    }
    publish(acc, part, fin, sh);
}

__global__ __launch_bounds__(kBlock) void k_cg_direction(int64_t n, double beta, double* __restrict__ p, const double* __restrict__ r) {
    NK_CHUNKED(i, n) p[i] = fma(beta, p[i], 1.0 * r[i]);
}

// ------------------------------------------------------------------------------ NK_USER pieces
// w = u + eps * (v / h) -- the same expression the fused FD stencils evaluate in registers -- and
// the normalised basis vector v / h (fused kdivcopy!), h = *vdiv on the device (1 when null).
__global__ __launch_bounds__(kBlock) void k_fd_point(int64_t n, double* __restrict__ w, const double* __restrict__ u,
                                                    const double* __restrict__ v, const double* __restrict__ vdiv,
                                                    double eps, double* __restrict__ vout) {
    const double hd = vdiv ? *vdiv : 1.0;
    NK_CHUNKED(i, n) {
        const double vi = vdiv ? v[i] / hd : v[i];
        if (w) w[i] = u[i] + eps * vi;
        if (vout) vout[i] = vi;
    }
}

// after a user F (FD: out = F(w)) or J: out = (out - F0) / eps (FD), then the stencil epilogue
template <int EPI>
__global__ __launch_bounds__(kBlock) void k_user_epi(int64_t n, int fd, double* __restrict__ out,
                                                    const double* __restrict__ F0, double eps,
                                                    const double* __restrict__ aux, double* __restrict__ part, int fin) {
    __shared__ double sh[kShN];
    double acc = 0.0;
    NK_CHUNKED(i, n) {
        double r = out[i];
        if (fd) r = (r - F0[i]) / eps;
        const double ax = (EPI == EPI_DOT || EPI == EPI_RESID) ? aux[i] : 0.0;
        acc = epilogue<EPI>(r, ax, acc);
        if (fd || EPI == EPI_RESID) out[i] = r;
    }
    if constexpr (EPI != EPI_NONE) publish(acc, part, fin, sh);
}

// ------------------------------------------------------------------------------ preconditioning
// z = d .* v (diagonal right preconditioner) with the partials of ||z||^2 (the FD step size)
__global__ __launch_bounds__(kBlock) void k_diag_apply(int64_t n, double* __restrict__ z, const double* __restrict__ d,
                                                      const double* __restrict__ v, double* __restrict__ part, int fin) {
    __shared__ double sh[kShN];
    double acc = 0.0;
    NK_CHUNKED(i, n) {
        const double zi = d[i] * v[i];
        z[i] = zi;
        acc = fma(zi, zi, acc);
    }
    if (part) publish(acc, part, fin, sh);
}

// diag(J(u)): the exact tangent at point i applied to the unit vector e_i -- the centre value 1,
// every neighbour 0 -- through the same lapk / point_value arithmetic as the stencil kernels
template <int KIND, int DIM>
__global__ __launch_bounds__(kBlock) void k_jdiag(KArgs A, double* __restrict__ out, int recip) {
    const int64_t n = A.nx * A.ny * A.nz;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        // G_Midpoint!'s stencil field is (1 - α) v: its centre (1 - α), the "- v" term 1
        const double c = scheme_of<KIND>() == 1 ? (1.0 - A.alpha) * 1.0 : 1.0;
        double lsum = lapk(A, c, 0.0, 0.0, A.hx2, A.ihx2);
        if (DIM >= 2) lsum = lsum + lapk(A, c, 0.0, 0.0, A.hy2, A.ihy2);
        if (DIM == 3) lsum = lsum + lapk(A, c, 0.0, 0.0, A.hz2, A.ihz2);
        const double uc = (KIND == NK_BRATU1D || KIND == NK_BRATU2D) ? A.u[i] : 0.0;
        bool rare_ = false;
        const double d = point_value<KIND, MODE_JEXACT>(A, c, lsum, uc, 0.0, 0.0, 1.0, 0.0, &NKX_T[0][0], rare_);
        out[i] = recip ? 1.0 / d : d;
    }
}

}  // namespace

// partial-sum slot of a reduction launch.  With an RCCL communicator the kernel also folds its
// partials in place (publish) and finish_reduction only has to all-reduce part[kRedCap - 1].  With
// the peer mailbox the producer only writes its partials; the CONSUMING kernel sums them and
// exchanges the per-rank sums (reduce_input), under a mailbox epoch allotted here.
unsigned next_mb_epoch(nk_ctx* c) {
    if (c->mb_epoch >= 0xffffu) c->mb_epoch = 0;  // 16-bit epochs 1 .. 65535 (0 never tags a value)
    return ++c->mb_epoch;
}

double* red_out(nk_ctx* c, int len, Red* r, int* fin) {
    double* part = red_slot(c);
    *fin = (c->comm && !c->mb_on) ? 1 : 0;
    r->epoch = 0;
    if (c->mb_on) r->epoch = next_mb_epoch(c);
    r->ptr = part;
    r->len = len;
    r->fin = *fin ? part + kRedCap - 1 : nullptr;
    return part;
}

// The binding (g_mb, one copy per translation unit and device) is process-wide: several contexts
// on one device share it.  A context binds its mailbox when it turns it on, and clears the binding
// only if it is the one bound -- tearing down a context without a mailbox (or another one's) must
// not unbind a live one.
namespace {
constexpr int kMaxDevices = 64;
nk_ctx* g_mb_owner[kMaxDevices] = {};
}  // namespace

int mailbox_bind(nk_ctx* c) {
    const int d = (c->device >= 0 && c->device < kMaxDevices) ? c->device : 0;
    if (!c->mb_on && g_mb_owner[d] != c) return NK_OK;
    g_mb_owner[d] = c->mb_on ? c : nullptr;
    MbInfo m{};
    if (c->mb_on) {
        m.self = c->mb_self;
        m.peers = c->mb_peers_dev;
        m.rank = c->rank;
        m.nranks = c->nranks;
        m.err = c->mb_err_dev;
        // polls before a mailbox wait gives up with an error (a few s: ranks may drift apart at start-up;
        // NK_MB_SPIN_LIMIT shortens it for the failure-path tests)
        const char* e = getenv("NK_MB_SPIN_LIMIT");
        m.spin_limit = (e && *e) ? (unsigned)atoll(e) : (1u << 26);
        if (!c->mb_wacc) {  // the peer-wait counters (nk_path_info), zeroed once per context
            NK_HIP(c, hipMalloc(reinterpret_cast<void**>(&c->mb_wacc), 4 * sizeof(unsigned long long)));
            NK_HIP(c, hipMemset(c->mb_wacc, 0, 4 * sizeof(unsigned long long)));
        }
        m.wacc = c->mb_wacc;
    }
    NK_HIP(c, hipMemcpyToSymbol(HIP_SYMBOL(g_mb), &m, sizeof(m)));
    // and the copy in every stencil instantiation unit
    for (auto bind : {stencil_bind_mb_1, stencil_bind_mb_2, stencil_bind_mb_3, stencil_bind_mb_4, stencil_bind_mb_5,
                      stencil_bind_mb_6, stencil_bind_mb_7, stencil_bind_mb_8, resident_bind_mb})
        NK_HIP(c, bind(m));
    return NK_OK;
}

namespace {
__global__ void k_mb_test(unsigned epoch, double value, double* out) {
    __shared__ double sh[kShN];
    mb_send(value, epoch);
    const double t = mb_recv(epoch, sh);
    if (threadIdx.x == 0) *out = t;
}
}  // namespace

namespace {

// Ghost planes through the peers' inboxes (IPC-mapped fine-grained memory over xGMI).  Block b
// owns chunk b of the plane: it pushes my boundary-plane chunks into the lower / upper
// neighbour's inbox (system-scope stores), drains, raises its epoch flag there, then waits for the
// neighbours' block b flags in my region and copies their chunks into my ghost planes.  Inboxes
// alternate by epoch parity: epoch e's push can only start after the neighbour finished epoch e-2.
// ring = 1 (bc_periodic! along the slab axis): rank 0's lower neighbour is rank nranks-1 and vice versa.
__global__ __launch_bounds__(kBlock) void k_halo_ipc(double* __restrict__ v, int64_t plane, int64_t nplanes,
                                                    uint64_t epoch, int64_t cap, int ring) {
    __shared__ int ready;
    const int b = blockIdx.x, rank = g_mb.rank, nr = g_mb.nranks;
    const bool lo = rank > 0 || ring, hi = rank + 1 < nr || ring;
    const int rlo = rank > 0 ? rank - 1 : nr - 1, rhi = rank + 1 < nr ? rank + 1 : 0;
    const int par = (int)(epoch & 1);
    const int64_t per = (plane + gridDim.x - 1) / gridDim.x;
    const int64_t c0 = (int64_t)b * per, c1 = c0 + per < plane ? c0 + per : plane;
    const double* first = v;
    const double* last = v + (nplanes - 1) * plane;
    if (lo) {  // my first interior plane -> the lower rank's "from upper" inbox
        uint64_t* dst = halo_inbox(g_mb.peers[rlo], par, 1, cap);
        for (int64_t i = c0 + threadIdx.x; i < c1; i += kBlock)
            __hip_atomic_store(dst + i, (uint64_t)__double_as_longlong(first[i]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (hi) {  // my last interior plane -> the upper rank's "from lower" inbox
        uint64_t* dst = halo_inbox(g_mb.peers[rhi], par, 0, cap);
        for (int64_t i = c0 + threadIdx.x; i < c1; i += kBlock)
            __hip_atomic_store(dst + i, (uint64_t)__double_as_longlong(last[i]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every thread drains its stores before the flag
    __syncthreads();
    if (threadIdx.x < 64) {  // lane 0 the lower side, lane 1 the upper: flags raised and polled in parallel
        const int side = (int)threadIdx.x;
        const bool mine = (side == 0 && lo) || (side == 1 && hi);
        if (mine)
            __hip_atomic_store(halo_flags(g_mb.peers[side == 0 ? rlo : rhi]) + (par * kHaloSides + (side ^ 1)) * kHaloBlocks + b,
                               epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t t0 = wall_clock64();
        const bool ok = !mine || flag_wait(halo_flags(g_mb.self) + (par * kHaloSides + side) * kHaloBlocks + b, epoch);
        const bool all = __all(ok);
        if (side == 0) {
            ready = all ? 1 : 0;
            wait_note(kWaitHalo, t0);
        }
    }
    __syncthreads();
    if (!ready) return;
    if (lo) {
        const uint64_t* src = halo_inbox(g_mb.self, par, 0, cap);
        for (int64_t i = c0 + threadIdx.x; i < c1; i += kBlock)
            v[i - plane] = __longlong_as_double((long long)__hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    }
    if (hi) {
        const uint64_t* src = halo_inbox(g_mb.self, par, 1, cap);
        for (int64_t i = c0 + threadIdx.x; i < c1; i += kBlock)
            v[nplanes * plane + i] =
                __longlong_as_double((long long)__hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    }
}

// 3D blocks (nk_dist_grid): the six ghost layers of v through the peers' inboxes in ONE launch (packed
// faces).  Block b owns chunk b of every face: it pushes my boundary layer on each side s that has a
// neighbour into that neighbour's inbox for side s ^ 1 (system-scope stores), drains, raises its flag
// there, waits for the neighbours' block-b flags in my region and unpacks their layers -- the z ones into
// my ghost planes, the x / y ones into the faces after the allocation's trailing plane.  Neighbours share
// the face's extents, and the grid size is a constant, so both sides cut a face alike.  At a
// physical boundary the layer stays zero (zero-filled allocation, never written there).
struct FaceArgs {
    int64_t nx, ny, nz;
    int64_t fy, fx;  // offsets of the y-lo / x-lo faces from the interior pointer
    int nbr[kHaloSides];
};
__device__ __forceinline__ int64_t face_len(const FaceArgs& F, int s) {
    return s < 2 ? F.nx * F.ny : (s < 4 ? F.nx * F.nz : F.ny * F.nz);
}
// element i of my boundary layer on side s: planes (k fastest-y-x order of a plane), y faces k nx + x,
// x faces k ny + j
__device__ __forceinline__ int64_t face_src(const FaceArgs& F, int s, int64_t i) {
    const int64_t pl = F.nx * F.ny;
    if (s == 0) return i;
    if (s == 1) return (F.nz - 1) * pl + i;
    if (s < 4) return (i / F.nx) * pl + (s == 2 ? 0 : F.ny - 1) * F.nx + i % F.nx;
    return (i / F.ny) * pl + (i % F.ny) * F.nx + (s == 4 ? 0 : F.nx - 1);
}
// where element i of the layer from side s lands in my allocation
__device__ __forceinline__ int64_t face_dst(const FaceArgs& F, int s, int64_t i) {
    const int64_t pl = F.nx * F.ny;
    if (s == 0) return i - pl;
    if (s == 1) return F.nz * pl + i;
    if (s < 4) return F.fy + (s == 3 ? F.nx * F.nz : 0) + i;
    return F.fx + (s == 5 ? F.ny * F.nz : 0) + i;
}
__global__ __launch_bounds__(kBlock) void k_faces_ipc(double* __restrict__ v, FaceArgs F, uint64_t epoch, int64_t cap) {
    __shared__ int ready;
    const int b = blockIdx.x, G = gridDim.x;
    const int par = (int)(epoch & 1);
    for (int s = 0; s < kHaloSides; ++s) {
        if (F.nbr[s] < 0) continue;
        const int64_t len = face_len(F, s), per = (len + G - 1) / G;
        const int64_t c0 = (int64_t)b * per, c1 = c0 + per < len ? c0 + per : len;
        uint64_t* dst = halo_inbox(g_mb.peers[F.nbr[s]], par, s ^ 1, cap);
        for (int64_t i = c0 + threadIdx.x; i < c1; i += kBlock)
            __hip_atomic_store(dst + i, (uint64_t)__double_as_longlong(v[face_src(F, s, i)]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every thread drains its stores before the flags
    __syncthreads();
    if (threadIdx.x < 64) {  // lane s raises side s's flag and polls its own: six round trips in parallel
        const int s = (int)threadIdx.x;
        int nbr = -1;
#pragma unroll
        for (int q = 0; q < kHaloSides; ++q)
            if (q == s) nbr = F.nbr[q];
        if (nbr >= 0)
            __hip_atomic_store(halo_flags(g_mb.peers[nbr]) + (par * kHaloSides + (s ^ 1)) * kHaloBlocks + b, epoch,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t t0 = wall_clock64();
        const bool ok = nbr < 0 || flag_wait(halo_flags(g_mb.self) + (par * kHaloSides + s) * kHaloBlocks + b, epoch);
        const bool all = __all(ok);
        if (s == 0) {
            ready = all ? 1 : 0;
            wait_note(kWaitHalo, t0);
        }
    }
    __syncthreads();
    if (!ready) return;
    for (int s = 0; s < kHaloSides; ++s) {
        if (F.nbr[s] < 0) continue;
        const int64_t len = face_len(F, s), per = (len + G - 1) / G;
        const int64_t c0 = (int64_t)b * per, c1 = c0 + per < len ? c0 + per : len;
        const uint64_t* src = halo_inbox(g_mb.self, par, s, cap);
        for (int64_t i = c0 + threadIdx.x; i < c1; i += kBlock)
            v[face_dst(F, s, i)] = __longlong_as_double((long long)__hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    }
}

// The per-tile partials of a one-shot stencil launch (more tiles than the next kernel should read
// partials) folded in groups of G tiles: block g sums tiles gG .. gG + G - 1 in tile order (lane l
// takes l, l + 64, ..., then a fixed wave tree) and hands the sum on as partial g -- with `fin` the
// last block also folds the partials, as the stencil itself would (publish_sum).  Bit-reproducible.
__global__ __launch_bounds__(64) void k_tile_fold(const double* __restrict__ tpart, int G, int ntiles, double* part,
                                                  int fin) {
    __shared__ double sh[kShN];
    const int g = blockIdx.x, g0 = g * G, m = (ntiles - g0) < G ? ntiles - g0 : G;
    double v = 0.0;
    for (int i = (int)threadIdx.x; i < m; i += 64) v += tpart[g0 + i];
    v = wave_sum(v);
    publish_sum<64>(v, part, fin, sh, g, (int)gridDim.x);
}

// bc_periodic! along the slab axis of a lone slab: ghost plane -1 <- the last interior plane,
// ghost plane nplanes <- the first (heat_2D.jl:20-21 / 23-24)
__global__ __launch_bounds__(kBlock) void k_periodic_fill(double* __restrict__ v, int64_t plane, int64_t nplanes) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < plane; i += (int64_t)gridDim.x * kBlock) {
        v[i - plane] = v[(nplanes - 1) * plane + i];
        v[nplanes * plane + i] = v[i];
    }
}
}  // namespace

int launch_halo_ipc(nk_ctx* c, double* v, int64_t plane, int64_t nplanes, bool ring) {
    if (halo_self_ring(c)) ring = true;
    else if (c->nranks < 2) return NK_OK;
    const uint64_t epoch = ++c->halo_epoch;
    static const int nb_env = std::max(1, std::min(kHaloBlocks, NK_TUNE("NK_HALO_NB", kHaloBlocks)));  // (kbench A/B)
    const int nb_max = std::min(nb_env, c->xchg_nb);
    int nb = (int)((plane + 1023) / 1024);
    if (nb > nb_max) nb = nb_max;
    if (nb < 1) nb = 1;
    const int nbrs = ring ? 2 : (c->rank > 0) + (c->rank + 1 < c->nranks);
    return launch(c, "halo_ipc", 16.0 * plane * nbrs, [&] {
        hipLaunchKernelGGL(k_halo_ipc, dim3(nb), dim3(kBlock), 0, c->stream, v, plane, nplanes, epoch, c->halo_cap,
                           ring ? 1 : 0);
    });
}

int launch_faces_ipc(nk_ctx* c, double* v, const nk_problem* p) {
    Geo g;
    NK_TRY(geometry(c, p, &g));
    FaceArgs F{};
    F.nx = p->nx;
    F.ny = p->ny;
    F.nz = p->nz;
    F.fy = g.n + g.plane;
    F.fx = F.fy + 2 * p->nx * p->nz;
    double bytes = 0.0;
    for (int s = 0; s < kHaloSides; ++s) {
        F.nbr[s] = block_nbr(c, s);
        if (F.nbr[s] >= 0) bytes += 16.0 * (double)(s < 2 ? p->nx * p->ny : (s < 4 ? p->nx * p->nz : p->ny * p->nz));
    }
    if (bytes == 0.0) return NK_OK;
    const uint64_t epoch = ++c->halo_epoch;
    // every rank cuts a face into the same nb chunks (xchg_nb is agreed at mailbox set-up, never the face's size)
    static const int nb_env = std::max(1, std::min(kHaloBlocks, NK_TUNE("NK_FACE_NB", kHaloBlocks)));  // (kbench A/B)
    const int nb = std::min(nb_env, c->xchg_nb);
    return launch(c, "halo_faces", bytes, [&] {
        hipLaunchKernelGGL(k_faces_ipc, dim3(nb), dim3(kBlock), 0, c->stream, v, F, epoch, c->halo_cap);
    });
}

int launch_periodic_fill(nk_ctx* c, double* v, int64_t plane, int64_t nplanes) {
    const int g = (int)std::min<int64_t>((plane + kBlock - 1) / kBlock, 1024);
    return launch(c, "periodic_fill", 16.0 * plane, [&] {
        hipLaunchKernelGGL(k_periodic_fill, dim3(g), dim3(kBlock), 0, c->stream, v, plane, nplanes);
    });
}

// every rank sends (rank + 1) (e + 1) for a few epochs; the sums must arrive exactly
int mailbox_selftest(nk_ctx* c, bool* ok) {
    *ok = true;
    for (int e = 0; e < 4; ++e) {
        const unsigned epoch = next_mb_epoch(c);
        hipLaunchKernelGGL(k_mb_test, dim3(1), dim3(64), 0, c->stream, epoch, (double)(c->rank + 1) * (e + 1), c->scal);
        NK_HIP(c, hipGetLastError());
        NK_HIP(c, hipMemcpyAsync(c->hpin, c->scal, sizeof(double), hipMemcpyDeviceToHost, c->stream));
        NK_HIP(c, hipStreamSynchronize(c->stream));
        const double want = (double)c->nranks * (c->nranks + 1) / 2 * (e + 1);
        if (c->hpin[0] != want || *c->mb_err) *ok = false;
    }
    return NK_OK;
}

// ghost planes of a Krylov Jv inside the stencil launch when the peer mailbox is up (kbench: NK_HALO_FUSE=0
// forces the separate exchange kernel)
int halo_fuse_knob() {
    static const int fuse = NK_TUNE("NK_HALO_FUSE", 1);
    return fuse;
}

// kbench only (NK_HALO_SELF=1, with a forced one-rank mailbox): the lone rank is its own lower and upper
// neighbour -- a self ring that runs the whole ghost-plane exchange on one GPU (tools/halo_self.py)
bool halo_self_ring(const nk_ctx* c) {
    static const int self = NK_TUNE("NK_HALO_SELF", 0);
    return self && c->mb_on && c->nranks == 1;
}
// kbench only (NK_HALO_SELF=2): the lone rank is its own neighbour on all six sides of a 3D block -- the
// packed-face exchange and k_st3l's face reads of config 5's blocks, timed on one GPU (tools/halo_self.py)
bool block_self(const nk_ctx* c) {
    static const int self = NK_TUNE("NK_HALO_SELF", 0);
    return self == 2 && c->mb_on && c->nranks == 1;
}

int red_blocks(int64_t n) {
    static const int cap = NK_TUNE("NK_RED_BLOCKS", kMaxRedBlocks);
    int64_t g = (n + 2LL * kBlock * 4 - 1) / (2LL * kBlock * 4);  // >= 4 double2 per thread
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

// Grid of the streaming kernels whose partials (if any) only a one-block finaliser reads: up to
// kRedCap - 2 blocks, >= 2 double2 per thread.  Many short-lived blocks stream faster than a
// grid of 8 per CU looping over block chunks (tools/stream_probe.py: a plain copy 5.0 -> 6.2 TB/s;
// k_update_x -9 % on heat 8192^2, profiles/r02/ab_redblocks.log).  Reductions consumed by every
// block of the next kernel (dot, sumsq, the MGS chain) keep red_blocks: each consumer block sums
// all the partials.
int wide_blocks(int64_t n) {
    static const int cap = std::max(1, std::min(kRedCap - 2, NK_TUNE("NK_WIDE_BLOCKS", kRedCap - 2)));
    int64_t g = (n + 2LL * kBlock * 2 - 1) / (2LL * kBlock * 2);
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

namespace {
int launch_stencil_ex(nk_ctx* c, const StencilIn& in, Red* red, int rows_override, int fast);
}

int launch_stencil(nk_ctx* c, const StencilIn& in, Red* red) {
    if (in.p && nk_is_user(in.p->kind)) {
        if (in.xchg_v) NK_TRY(halo_exchange(c, in.p, in.v));
        return launch_user(c, in, red);
    }
    return launch_stencil_ex(c, in, red, 0, 0);
}

namespace {
int launch_stencil_ex(nk_ctx* c, const StencilIn& in, Red* red, int rows_override, int fast) {
    const nk_problem* p = in.p;
    Geo g;
    NK_TRY(geometry(c, p, &g));
    KArgs A{};
    A.out = in.out; A.u = in.u; A.v = in.v; A.F0 = in.F0; A.un = p->un; A.aux = in.aux;
    A.nx = p->nx; A.ny = p->ny; A.nz = p->nz;
    A.hx2 = p->hx * p->hx; A.hy2 = p->hy * p->hy; A.hz2 = p->hz * p->hz;
    A.lam = p->lambda; A.a = p->a; A.dt = p->dt; A.eps = in.eps;
    // kbench A/B bits: 2^20 the platform exp, 2^22 the exp's fast phase alone (diagnosis: not correctly
    // rounded), 2^23 the Bratu stencils' divisions as division instruction sequences instead of div_rn
    A.fast = fast | (NK_TUNE("NK_EXP_OCML", 0) ? (1 << 20) : 0) | (NK_TUNE("NK_EXP_FASTONLY", 0) ? (1 << 22) : 0) |
             (NK_TUNE("NK_DIV_INSN", 0) ? (1 << 23) : 0);
    A.vdiv = in.vdiv;
    A.vout = in.vout;
    A.ihx2 = 1.0 / A.hx2; A.ihy2 = 1.0 / A.hy2; A.ihz2 = 1.0 / A.hz2; A.ieps = in.eps != 0.0 ? 1.0 / in.eps : 0.0;
    A.alpha = p->alpha;
    const bool per = p->bc == NK_BC_PERIODIC;
    int vec = 1, grid = 1;
    if (g.dim == 1) {
        grid = (int)((p->nx + kBlock - 1) / kBlock);
    } else if (g.dim == 2) {
        static const int vec_pref = NK_TUNE("NK_ST_VEC", 2);
        vec = (p->nx % 2 == 0) ? 2 : 1;
        if (((fast & 4) || vec_pref == 4) && p->nx % 4 == 0 && !per) vec = 4;
        A.tiles_x = (int)((p->nx + kBlock * vec - 1) / (kBlock * vec));
        // rows per tile: about 1024 tiles, between 8 and 32 rows (4096^2: 32-row tiles, FD Jv 121.3 ->
        // 114.8 us and +0.6 % on the bench, profiles/r02/ab_st_blocks.log; 8192^2 heat: 32 rows are
        // as fast as 64 for the FD Jv and 3 % faster for the residual, kbench_st2d_8192.log), and
        // never more tiles than the reduction slot holds partials
        static const int target = NK_TUNE("NK_ST_BLOCKS", 1024);
        int64_t rows = (p->ny * A.tiles_x + target - 1) / target;
        static const int min_rows = NK_TUNE("NK_ST_MINROWS", 8);
        static const int max_rows = NK_TUNE("NK_ST_MAXROWS", 32);
        if (rows > max_rows) rows = max_rows;
        if (rows < min_rows) rows = min_rows;
        const int64_t cap_rows = (p->ny * A.tiles_x + (kRedCap - 3)) / (kRedCap - 2);
        if (rows < cap_rows) rows = cap_rows;
        if (rows_override > 0) rows = rows_override;
        if (rows > p->ny) rows = p->ny;
        A.rows = (int)rows;
        A.tiles_y = (int)((p->ny + rows - 1) / rows);
        grid = A.tiles_x * A.tiles_y;
        A.lin = (fast & 2048) ? 1 : 0;  // kbench: tiles in address order
        // kbench only: one-shot LDS tiles (k_st2t: 8 rows x 128 columns, no march, tiles in address
        // order, block partials folded by k_tile_fold) for the FD operator (NK_ST_ONESHOT=1), or for any
        // mode with fast bits 8192 / 16384 / 32768 (8 / 4 / 16 rows); 262144 forces the march.  8-12 %
        // faster than the march in isolation (profiles/r03/ab_tile8.log, ab_oneshot_fold2.log), but not in
        // the bench (ab_oneshot4.log): the product keeps the march.
        static const int oneshot_env = NK_TUNE("NK_ST_ONESHOT", 0);
        A.tile2 = (fast & 8192) ? 8 : ((fast & 16384) ? 4 : ((fast & 32768) ? 16 : 0));
        if (!A.tile2 && oneshot_env && in.mode == MODE_JFD && vec == 2 && !(fast & (262144 | 4 | 2048)) &&
            rows_override <= 0 && !(oneshot_env == 2 && nk_scheme(p->kind) == 2))
            A.tile2 = 8;
        // fast bit 131072 with a one-shot tile: 256 columns wide (VEC 4), 8 or 4 rows
        if (A.tile2 && (fast & 131072) && p->nx % 4 == 0 && !per && !(A.tile2 == 16)) {
            vec = 4;
            A.tiles_x = (int)((p->nx + 255) / 256);
            A.tiles_y = (int)((p->ny + A.tile2 - 1) / A.tile2);
            grid = A.tiles_x * A.tiles_y;
        } else if (A.tile2 && vec == 2) {
            const int tx1 = (int)((p->nx + 127) / 128), ty1 = (int)((p->ny + A.tile2 - 1) / A.tile2);
            if ((int64_t)tx1 * ty1 <= kTileCap) {
                A.tiles_x = tx1;
                A.tiles_y = ty1;
                grid = A.tiles_x * A.tiles_y;
            } else {
                A.tile2 = 0;  // beyond the per-tile partial buffer: the row march
            }
        } else {
            A.tile2 = 0;
        }
    } else {
        vec = (p->nx % 2 == 0) ? 2 : 1;
        if (blocks3d(c, g)) {  // 3D blocks: x / y ghost layers from the faces after the trailing plane
            A.blk = 1;
            A.fy = g.n + g.plane;
            A.fx = A.fy + 2 * p->nx * p->nz;
            for (int sd = 2; sd < kHaloSides; ++sd)
                if (block_nbr(c, sd) >= 0) A.nbm |= 1 << sd;
        }
        // rows per 3D tile and the y-neighbour path (k_st3d loads, k_st3l LDS); fast bits 8 / 16 select
        // k_st3l with 4 / 8 rows (kernel-variant bench), NK_ST3_LDS / NK_ST3_NW likewise
        // k_st3l with 4-row tiles is the default: +6-16 % over k_st3d on every 3D kind / mode at 512^3
        // and at config 5's 512^2 x 64 slab (profiles/r02/kbench_st3l.log)
        static const int lds_env = NK_TUNE("NK_ST3_LDS", 1);
        static const int nw_env = NK_TUNE("NK_ST3_NW", 4);
        A.lds3 = (fast & 24) ? 1 : lds_env;
        A.nw = A.lds3 ? ((fast & 8) ? 4 : ((fast & 16) ? 8 : (nw_env == 4 ? 4 : 8))) : 4;
        if (A.blk) {  // 3D blocks: k_st3l with 4-row tiles (the kernel-variant build's other forms have no faces)
            A.lds3 = 1;
            A.nw = 4;
        }
        A.tiles_x = (int)((p->nx + 64 * vec - 1) / (64 * vec));
        A.tiles_y = (int)((p->ny + A.nw - 1) / A.nw);
        static const int target = NK_TUNE("NK_ST3_BLOCKS", 8192);  // shorter z-marches keep y-adjacent tiles in step (L2 reuse of the halo rows)
        int64_t planes = ((int64_t)p->nz * A.tiles_x * A.tiles_y + target - 1) / target;
        static const int min_planes = NK_TUNE("NK_ST_MINPLANES", 16);  // 16: (16 + 2) / 16 z-halo re-reads
        if (planes < min_planes) planes = min_planes;
        if (rows_override > 0) planes = rows_override;
        if (planes > p->nz) planes = p->nz;
        A.rows = (int)planes;
        grid = A.tiles_x * A.tiles_y * (int)((p->nz + planes - 1) / planes);
        // k_st3l tile order / march direction (tile3_of; kbench only: 1 whole tile columns per XCD band with
        // odd z-chunks marching down, 2 plane-major + odd chunks down, 3 chunk pairs): within +-3 % of the
        // plane-major order, upward marches (0, the product) -- profiles/r03/ab_zalt*.log
        static const int zalt_env = NK_TUNE("NK_ST3_ZALT", 0);
        A.zalt = (A.lds3 && !(fast & 65536) && !A.blk) ? zalt_env : 0;  // kbench fast bit 65536: the plane-major order
        // the y-march (k_st3y, kbench NK_ST3_YMARCH=1: slabs short along z; NK_ST3Y_ROWS rows per chunk):
        // tiles of nw planes x 64 vec columns marching a chunk of rows
        static const int ym_env = NK_TUNE("NK_ST3_YMARCH", 0);
        static const int ym_rows = NK_TUNE("NK_ST3Y_ROWS", 64);
        A.ym = (A.lds3 && (ym_env || (fast & 524288)) && rows_override <= 0 && !A.zalt && !A.blk) ? 1 : 0;  // (bit 2^19: the y-march)
        if (A.ym) {
            const int64_t r = std::min<int64_t>(std::max(1, ym_rows), p->ny);
            A.rows = (int)r;
            A.tiles_y = (int)((p->ny + r - 1) / r);
            grid = A.tiles_x * A.tiles_y * (int)((p->nz + A.nw - 1) / A.nw);
        }
    }
    // FD with F0 recomputed from u (2D, VEC <= 2: k_st2d<..., F0R>; 3D heat: k_st3l<..., F0R>, not
    // with NK_F0R=3 (A/B)); never with the `fast` reciprocals,
    // which would change F(u) against the residual kernel that stored F0.  NK_F0R: 1 (default) for the
    // heat kinds, whose F(u) costs a few flops (8192^2 FD Jv 728 -> 612 us, bench +3.3 %), and for
    // Bratu's Jv launches that also store V_k (fused normalisation): they move enough bytes to hide the
    // second exp per point (config-4 slab Jv 277 -> 246 us, V_1 step 248 -> 227 us, bench +1.2 %),
    // while the plain Jv + dot (116 -> 122 us) and the restart residual (110 -> 126 us) do not
    // (profiles/r02/ab_f0r_bratu.log); 2 for every Bratu launch too; 0 never
#ifndef NK_F0R_DEFAULT  // (product variant builds for A/B: 0 never, 2 every FD launch, 3 no 3D F0R)
#define NK_F0R_DEFAULT 1
#endif
    static const int f0r_env = NK_TUNE("NK_F0R", NK_F0R_DEFAULT);
    // 3D: the F0R kernel needs 145 VGPRs (3 waves per SIMD instead of 4), which pays only where the
    // field is cheap and the kernel moves the most bytes: G_Euler!'s Jv with a dot partner (512^3
    // FD Jv + V_k store 1400 -> 1198 us), not the V_1 = r0 / beta step, not midpoint / trapezoid
    // (profiles/r02/ab_f0r3.log)
    const bool dotvs = in.vout && in.epi == EPI_DOT && !in.aux;
    const bool vfused = in.vout && in.epi == EPI_DOT;
    const bool f0r = f0r_env && in.f0r && in.mode == MODE_JFD && vec <= 2 && !(fast & 1) &&
                     ((g.dim == 2 && (f0r_env >= 2 || nk_is_heat(p->kind) || vfused)) ||
                      (g.dim == 3 && A.lds3 && f0r_env != 3 && (f0r_env >= 2 || (p->kind == NK_HEAT3D_EULER && !dotvs))));
    A.f0r = f0r ? 1 : 0;
    if (in.xchg_v) {
        // v's ghost planes: through the peers' inboxes inside this launch (halo_tile_exchange: only the
        // tiles at the slab's ends fetch, the rest of the grid never waits) when the peer mailbox is up,
        // the slab axis is not periodic and every tile of a plane has a flag; else exchanged first
        const int fuse_env = halo_fuse_knob();
        const int64_t tiles_pl = g.dim == 2 ? A.tiles_x : (int64_t)A.tiles_x * A.tiles_y;
        const bool self = halo_self_ring(c);
        // ranks sharing one GPU (rehearsals): in-launch only for small slabs -- a big slab's end tiles spin
        // on CUs the peer's producing tiles need (r05: 8 ranks x 256^2 x 32 planes, 30 s per step fused
        // against 27 ms with the exchange kernel, profiles/r05/rehearsal8_heat3d_256_*.json)
        const bool share_ok = c->res_share <= 1 || g.n <= kSharedFuseMax;
        const bool fuse = fuse_env && c->mb_on && (c->nranks > 1 || self) && share_ok && !per && !A.blk && in.mode != MODE_RES &&
                          (g.dim == 2 || (g.dim == 3 && A.lds3)) && g.plane <= c->halo_cap && tiles_pl <= kHaloTileFlags;
        if (fuse) {
            ++c->n_jv_halo_fused;
            A.hx_lo = c->rank > 0 || self;
            A.hx_hi = c->rank + 1 < c->nranks || self;
            A.hx_epoch = ++c->halo_epoch;
            A.hx_cap = c->halo_cap;
        } else {
            if (c->nranks > 1 || per) ++c->n_jv_halo_separate;
            NK_TRY(halo_exchange(c, p, in.v));
        }
    }
    if (in.epi != EPI_NONE) {
        int nparts = grid;
        A.group = 1;
        static const int tile_parts = std::max(1, std::min(kRedCap - 2, NK_TUNE("NK_TILE_PARTS", kTileParts)));
        if (A.tile2 && grid > tile_parts) {  // one-shot tiles: about kTileParts group partials handed on
            A.group = (grid + tile_parts - 1) / tile_parts;
            nparts = (grid + A.group - 1) / A.group;
            if (!c->tpart && hipMalloc(&c->tpart, sizeof(double) * (size_t)kTileCap) != hipSuccess)
                return fail(c, NK_E_NOMEM, "one-shot tile partials");
            A.tpart = c->tpart;
        }
        if (nparts > kRedCap - 2) return fail(c, NK_E_ARG, "stencil grid exceeds reduction capacity");
        A.part = red_out(c, nparts, red, &A.fin);
    }
    // algorithmic (compulsory) bytes per launch, for the instantiation the dispatch launched (StInst: an
    // F0R kernel reads no F0)
    const bool heat = nk_is_heat(p->kind);
    auto bytes_of = [&](const StInst& st) {
        int words = 1;  // out
        if (in.mode == MODE_RES) words += 1 + (heat ? 1 : 0);
        else if (in.mode == MODE_JEXACT) words += 1 + (heat ? 0 : 1);
        else words += 3 + (heat ? 1 : 0) - (st.f0r ? 1 : 0);
        if (in.epi == EPI_RESID || (in.epi == EPI_DOT && in.aux)) words += 1;
        if (in.vout) words += 1;  // fused kdivcopy!: V_k is written
        return 8.0 * words * (double)g.n;
    };
    static const char* names[3][4] = {
        {"residual", "residual_norm", "residual_dot", "residual_resid"},
        {"jv_exact", "jv_exact_sumsq", "jv_exact_dot", "jv_exact_resid"},
        {"jv_fd", "jv_fd_sumsq", "jv_fd_dot", "jv_fd_resid"}};
    static const char* fused_names[3] = {"residual", "jv_exact_dot_norm", "jv_fd_dot_norm"};
    static const char* v1_names[3] = {"residual", "jv_exact_dot_v1", "jv_fd_dot_v1"};
    if (in.vout && in.epi != EPI_DOT) return fail(c, NK_E_ARG, "fused normalisation needs the dot epilogue");
    // the kernels divide by h only in their V_k-storing instantiations (EPI_DOTV / EPI_DOTVS)
    if (in.vdiv && !in.vout) return fail(c, NK_E_ARG, "v / h is applied only with V_k stored (vout)");
    const int kind = p->kind, mode = in.mode;
    // distinct instantiations (own profile lines): normalise-and-store V_k, and its V_1 = r0/beta form
    // whose dot partner is the stored vector itself
    const int epi = (in.vout && in.epi == EPI_DOT) ? (in.aux ? EPI_DOTV : EPI_DOTVS) : in.epi;
    if (in.epi == EPI_DOT && !in.aux && !in.vout) return fail(c, NK_E_ARG, "dot epilogue needs its partner");
    hipStream_t s = c->stream;
    const char* kname = epi == EPI_DOTV ? fused_names[mode] : (epi == EPI_DOTVS ? v1_names[mode] : names[mode][epi]);
    StInst st{};
    const char* stname = st.name;
    const int rc = launch_dyn(c, kname, [&] {
        switch (kind) {  // one translation unit per kind (nk_stencil_inst.hip)
        case NK_BRATU1D: st = stencil_kind_1(A, mode, epi, vec, grid, s, false); break;
        case NK_BRATU2D: st = stencil_kind_2(A, mode, epi, vec, grid, s, false); break;
        case NK_HEAT2D_EULER: st = stencil_kind_3(A, mode, epi, vec, grid, s, per); break;
        case NK_HEAT3D_EULER: st = stencil_kind_4(A, mode, epi, vec, grid, s, per); break;
        case NK_HEAT2D_MIDPOINT: st = stencil_kind_5(A, mode, epi, vec, grid, s, per); break;
        case NK_HEAT3D_MIDPOINT: st = stencil_kind_6(A, mode, epi, vec, grid, s, per); break;
        case NK_HEAT2D_TRAPEZOID: st = stencil_kind_7(A, mode, epi, vec, grid, s, per); break;
        default: st = stencil_kind_8(A, mode, epi, vec, grid, s, per); break;
        }
        if (A.group > 1) {  // one-shot tiles: the group sums in tile order, as the next kernel's partials
            const int ng = (grid + A.group - 1) / A.group;
            hipLaunchKernelGGL(k_tile_fold, dim3(ng), dim3(64), 0, s, A.tpart, A.group, grid, A.part, A.fin);
        }
        return bytes_of(st);
    }, -1.0, &stname);
    if (rc == NK_OK && mode == MODE_JFD) ++(st.f0r ? c->n_fd_f0r : c->n_fd_f0_read);
    return rc;
}
}  // namespace

int launch_dot(nk_ctx* c, int64_t n, const double* x, const double* y, Red* red) {
    const int g = red_blocks(n);
    int fin;
    double* part = red_out(c, g, red, &fin);
    return launch(c, "dot", 16.0 * n, [&] { hipLaunchKernelGGL(k_dot, dim3(g), dim3(kBlock), 0, c->stream, n, x, y, part, fin); });
}

int launch_sumsq(nk_ctx* c, int64_t n, const double* x, Red* red) {
    const int g = red_blocks(n);
    int fin;
    double* part = red_out(c, g, red, &fin);
    return launch(c, "norm", 8.0 * n, [&] { hipLaunchKernelGGL(k_sumsq, dim3(g), dim3(kBlock), 0, c->stream, n, x, part, fin); });
}

int launch_finalize(nk_ctx* c, Red r, double* dst, int sqrt_it, double* mirror) {
    return launch(c, "finalize", 0.0,
                  [&] { hipLaunchKernelGGL(k_finalize, dim3(1), dim3(kBlock), 0, c->stream, r.ptr, r.len, dst, sqrt_it, mirror); });
}

#define NK_STREAM_LAUNCH(name, bytes_per, kern, ...)                                              \
    const int g = wide_blocks(n);                                                                  \
    return launch(c, name, (bytes_per) * (double)n,                                                \
                  [&] { hipLaunchKernelGGL(kern, dim3(g), dim3(kBlock), 0, c->stream, __VA_ARGS__); })

int launch_axpy(nk_ctx* c, int64_t n, double s, const double* x, double* y) { NK_STREAM_LAUNCH("axpy", 24.0, k_axpy, n, s, x, y); }
int launch_axpy_sumsq(nk_ctx* c, int64_t n, double s, const double* x, double* y, Red* red) {
    const int g = red_blocks(n);
    int fin;
    double* part = red_out(c, g, red, &fin);
    return launch(c, "axpy_norm", 24.0 * n,
                  [&] { hipLaunchKernelGGL(k_axpy_sumsq, dim3(g), dim3(kBlock), 0, c->stream, n, s, x, y, part, fin); });
}
int launch_axpby(nk_ctx* c, int64_t n, double s, const double* x, double t, double* y) {
    NK_STREAM_LAUNCH("axpby", 24.0, k_axpby, n, s, x, t, y);
}
int launch_scal(nk_ctx* c, int64_t n, double s, double* x) { NK_STREAM_LAUNCH("scal", 16.0, k_scal, n, s, x); }
int launch_copy(nk_ctx* c, int64_t n, double* y, const double* x) { NK_STREAM_LAUNCH("copy", 16.0, k_copy, n, y, x); }
int launch_fill(nk_ctx* c, int64_t n, double* x, double v) { NK_STREAM_LAUNCH("fill", 8.0, k_fill, n, x, v); }
int launch_divcopy(nk_ctx* c, int64_t n, double* y, const double* x, double s) {
    NK_STREAM_LAUNCH("divcopy", 16.0, k_divcopy, n, y, x, s);
}
int launch_ref(nk_ctx* c, int64_t n, double* x, double* y, double cc, double ss) { NK_STREAM_LAUNCH("ref", 32.0, k_ref, n, x, y, cc, ss); }
int launch_exp(nk_ctx* c, int64_t n, double* y, const double* x) { NK_STREAM_LAUNCH("exp", 16.0, k_exp, n, y, x); }

namespace {
template <bool HAS_NEXT>
void mgs_dispatch(int variant, int g, hipStream_t s, int64_t n, double* q, const double* vi, const double* vn,
                  const double* red, int len, double* h, double* hm, double* part, int rev, int fin) {
    switch (variant) {  // unroll depth x non-temporal V_i loads (tools/kbench.py measures them)
#ifdef NK_KBENCH
    case 0: hipLaunchKernelGGL((k_mgs_pass<HAS_NEXT, 2, false>), dim3(g), dim3(kBlock), 0, s, n, q, vi, vn, red, len, h, hm, part, rev, fin); break;
    case 1: hipLaunchKernelGGL((k_mgs_pass<HAS_NEXT, 2, true>), dim3(g), dim3(kBlock), 0, s, n, q, vi, vn, red, len, h, hm, part, rev, fin); break;
    case 2: hipLaunchKernelGGL((k_mgs_pass<HAS_NEXT, 4, true>), dim3(g), dim3(kBlock), 0, s, n, q, vi, vn, red, len, h, hm, part, rev, fin); break;
    case 3: hipLaunchKernelGGL((k_mgs_pass<HAS_NEXT, 2, true, true>), dim3(g), dim3(kBlock), 0, s, n, q, vi, vn, red, len, h, hm, part, rev, fin); break;
    case 4: hipLaunchKernelGGL((k_mgs_pass<HAS_NEXT, 4, true, true>), dim3(g), dim3(kBlock), 0, s, n, q, vi, vn, red, len, h, hm, part, rev, fin); break;
    case 6: hipLaunchKernelGGL((k_mgs_pass<HAS_NEXT, 4, true, false, true>), dim3(g), dim3(kBlock), 0, s, n, q, vi, vn, red, len, h, hm, part, rev, fin); break;
    case 7: hipLaunchKernelGGL((k_mgs_pass<HAS_NEXT, 2, true, true, true>), dim3(g), dim3(kBlock), 0, s, n, q, vi, vn, red, len, h, hm, part, rev, fin); break;
#endif
    case 5: hipLaunchKernelGGL((k_mgs_pass<HAS_NEXT, 2, true, false, true>), dim3(g), dim3(kBlock), 0, s, n, q, vi, vn, red, len, h, hm, part, rev, fin); break;
    default: hipLaunchKernelGGL((k_mgs_pass<HAS_NEXT, 2, true, true, true, true>), dim3(g), dim3(kBlock), 0, s, n, q, vi, vn, red, len, h, hm, part, rev, fin); break;
    }
}

}  // namespace
int launch_mgs_pass(nk_ctx* c, int64_t n, double* q, const double* vi, const double* vnext, Red in, double* h_out,
                    double* h_host, Red* out,
                    int rev) {
    // vectors that fit the 256 MB Infinity Cache twice over (q + V_{i+1} re-read by the next pass):
    // cached q / V_{i+1} (variant 5); larger ones stream every operand non-temporally (variant 8:
    // +1.8 % heat 8192^2, +2.3 % heat 512^3; it costs 16 % at 4096^2)
    static const int forced = NK_TUNE("NK_MGS_VARIANT", -1);
    const int variant = forced >= 0 ? forced : (8.0 * (double)n > 256.0 * (1 << 20) ? 8 : kMgsVariant);
    const int g = red_blocks(n);
    int fin;
    double* part = red_out(c, g, out, &fin);
    ++c->n_mgs_pass;
    if (vnext)
        // unique-DRAM model: V_{i+1} is the next pass's V_i (counted there), so q in + q out + V_i
        return launch(c, "mgs_pass", 32.0 * n, [&] {
            mgs_dispatch<true>(variant, g, c->stream, n, q, vi, vnext, in.ptr, in.len, h_out, h_host, part, rev, fin);
        }, 24.0 * n);
    return launch(c, "mgs_pass_last", 24.0 * n, [&] {
        mgs_dispatch<false>(variant, g, c->stream, n, q, vi, vnext, in.ptr, in.len, h_out, h_host, part, rev, fin);
    });
}

int launch_update_x(nk_ctx* c, int64_t n, double* x, double* xr, const double* const* V, int k, const double* y_dev,
                    int restart, Red* xnorm, double* u) {
    const int g = wide_blocks(n);  // its ||x|| / ||u|| partials go to the finaliser only
    int done = 0;
    if (k == 0) {  // nothing to add: x unchanged (restart) or x = 0
        if (!restart) NK_TRY(launch_fill(c, n, x, 0.0));
        if (u) return launch_axpy_sumsq(c, n, -1.0, x, u, xnorm);
        if (xnorm) return launch_sumsq(c, n, x, xnorm);
        return NK_OK;
    }
    while (done < k) {
        UpdArgs A{};
        static const int cap = std::max(1, std::min(kMaxUpdateVecs, NK_TUNE("NK_UPD_VECS", kMaxUpdateVecs)));
        const int m = (k - done) < cap ? (k - done) : cap;
        for (int i = 0; i < m; ++i) A.V[i] = V[done + i];
        A.x = x; A.xr = xr; A.y = y_dev + done; A.n = n; A.k = m;
        A.first = done == 0;
        A.last = done + m == k;
        A.restart = restart;
        A.u = A.last ? u : nullptr;
        A.part = nullptr;
        if (A.last && xnorm) A.part = red_out(c, g, xnorm, &A.fin);
        // every chunk reads m basis vectors and (after the first) xr; the last writes x (reading it on restart)
        const double bytes = 8.0 * n * (m + (A.first ? 0 : 1) + (A.last ? (restart ? 2 : 1) + (u ? 1 : 0) : 1));
        // 4 elements per thread and iteration: +10-25 % over 1 for every chain length k = 1..30 at
        // 4096^2 and 8192^2 (profiles/r02/kbench_upd.log); NK_UPD_U = 1 / 2 / 8 for A/B
#ifdef NK_KBENCH
        static const int uenv = NK_TUNE("NK_UPD_U", 0);
        const int U = uenv > 0 ? uenv : 4;
#endif
        NK_TRY(launch(c, "update_x", bytes, [&] {
#ifdef NK_KBENCH
            if (U >= 8) hipLaunchKernelGGL(k_update_x<8>, dim3(g), dim3(kBlock), 0, c->stream, A);
            else if (U == 2) hipLaunchKernelGGL(k_update_x<2>, dim3(g), dim3(kBlock), 0, c->stream, A);
            else if (U == 1) hipLaunchKernelGGL(k_update_x<1>, dim3(g), dim3(kBlock), 0, c->stream, A);
            else
#endif
                hipLaunchKernelGGL(k_update_x<4>, dim3(g), dim3(kBlock), 0, c->stream, A);
        }));
        done += m;
    }
    return NK_OK;
}

int launch_cg_update(nk_ctx* c, int64_t n, double alpha, double* x, double* r, const double* p, const double* Ap, Red* rr) {
    const int g = red_blocks(n);
    int fin;
    double* part = red_out(c, g, rr, &fin);
    return launch(c, "cg_update", 48.0 * n, [&] {
        hipLaunchKernelGGL(k_cg_update, dim3(g), dim3(kBlock), 0, c->stream, n, alpha, x, r, p, Ap, part, fin);
    });
}

int launch_fd_point(nk_ctx* c, int64_t n, double* w, const double* u, const double* v, const double* vdiv,
                    double eps, double* vout) {
    NK_STREAM_LAUNCH("user_fd_point", 8.0 * (1 + (w ? 2 : 0) + (vout ? 1 : 0)), k_fd_point, n, w, u, v, vdiv, eps, vout);
}

int launch_user_epi(nk_ctx* c, int64_t n, int fd, double* out, const double* F0, double eps, int epi, const double* aux,
                    Red* red) {
    const int g = red_blocks(n);
    int fin = 0;
    double* part = nullptr;
    if (epi != EPI_NONE) part = red_out(c, g, red, &fin);
    const double words = 1 + (fd ? 2 : 0) + ((epi == EPI_DOT || epi == EPI_RESID) ? 1 : 0) + (epi == EPI_RESID ? 1 : 0);
    return launch(c, "user_epilogue", 8.0 * words * n, [&] {
        switch (epi) {
        case EPI_NONE: hipLaunchKernelGGL(k_user_epi<EPI_NONE>, dim3(g), dim3(kBlock), 0, c->stream, n, fd, out, F0, eps, aux, part, fin); break;
        case EPI_SUMSQ: hipLaunchKernelGGL(k_user_epi<EPI_SUMSQ>, dim3(g), dim3(kBlock), 0, c->stream, n, fd, out, F0, eps, aux, part, fin); break;
        case EPI_DOT: hipLaunchKernelGGL(k_user_epi<EPI_DOT>, dim3(g), dim3(kBlock), 0, c->stream, n, fd, out, F0, eps, aux, part, fin); break;
        default: hipLaunchKernelGGL(k_user_epi<EPI_RESID>, dim3(g), dim3(kBlock), 0, c->stream, n, fd, out, F0, eps, aux, part, fin); break;
        }
    });
}

int launch_diag_apply(nk_ctx* c, int64_t n, double* z, const double* d, const double* v, Red* red) {
    const int g = red_blocks(n);
    int fin = 0;
    double* part = red ? red_out(c, g, red, &fin) : nullptr;
    return launch(c, "precond_diag", 24.0 * n, [&] {
        hipLaunchKernelGGL(k_diag_apply, dim3(g), dim3(kBlock), 0, c->stream, n, z, d, v, part, fin);
    });
}

int launch_jdiag(nk_ctx* c, const nk_problem* p, double* out, const double* u, int recip) {
    KArgs A{};
    A.u = u;
    A.nx = p->nx; A.ny = p->ny; A.nz = p->nz;
    A.hx2 = p->hx * p->hx; A.hy2 = p->hy * p->hy; A.hz2 = p->hz * p->hz;
    A.lam = p->lambda; A.a = p->a; A.dt = p->dt; A.alpha = p->alpha;
    const int64_t n = p->nx * p->ny * p->nz;
    const int g = (int)std::min<int64_t>((n + kBlock - 1) / kBlock, 4096);
#define NK_JDIAG(K, D) hipLaunchKernelGGL((k_jdiag<K, D>), dim3(g), dim3(kBlock), 0, c->stream, A, out, recip)
    return launch(c, "jacobian_diag", 16.0 * n, [&] {
        switch (p->kind) {
        case NK_BRATU1D: NK_JDIAG(NK_BRATU1D, 1); break;
        case NK_BRATU2D: NK_JDIAG(NK_BRATU2D, 2); break;
        case NK_HEAT2D_EULER: NK_JDIAG(NK_HEAT2D_EULER, 2); break;
        case NK_HEAT2D_MIDPOINT: NK_JDIAG(NK_HEAT2D_MIDPOINT, 2); break;
        case NK_HEAT2D_TRAPEZOID: NK_JDIAG(NK_HEAT2D_TRAPEZOID, 2); break;
        case NK_HEAT3D_MIDPOINT: NK_JDIAG(NK_HEAT3D_MIDPOINT, 3); break;
        case NK_HEAT3D_TRAPEZOID: NK_JDIAG(NK_HEAT3D_TRAPEZOID, 3); break;
        default: NK_JDIAG(NK_HEAT3D_EULER, 3); break;
        }
    });
#undef NK_JDIAG
}

// ------------------------------------------------------------------------------ ILU(0)
// ILU(0) of the stencil Jacobian in natural order (x fastest) -- the `N = (J) -> ilu(collect(J))` of
// examples/bratu.jl:119-137 restricted to J's own sparsity pattern.  For 3/5/7-point stencils the
// IKJ elimination only updates the diagonal (no pattern entry of a lower neighbour is an upper
// neighbour of another), so the factor is L = I + L_A D~^-1, U = D~ + U_A with
//   D~_i = ((a_ii - (c_z / D~_b) c_z) - (c_y / D~_s) c_y) - (c_x / D~_w) c_x     (lower neighbours in
// increasing index order: below, south, west; c_* = the constant off-diagonals of J).  Point i
// depends on its lower neighbours only, so every anti-diagonal level x + y + z = L is independent:
// one work-group sweeps the levels with a barrier in between (the same arithmetic, in the same
// order per point, as the oracle's sequential loop -- bit-identical).  A block-Jacobi factor when
// distributed: each slab is factored on its own (no ghost couplings).
struct IluArgs {
    int64_t nx, ny, nz;
    double cx, cy, cz;  // off-diagonal entries of J along x, y, z
};

template <typename F>
__device__ __forceinline__ void ilu_levels(const IluArgs& I, bool reverse, F&& f) {
    const int64_t nlev = (I.nx - 1) + (I.ny - 1) + (I.nz - 1) + 1;
    const int64_t nyz = I.ny * I.nz;
    for (int64_t t = 0; t < nlev; ++t) {
        const int64_t L = reverse ? nlev - 1 - t : t;
        // the (y, z) pairs whose x = L - y - z lies in [0, nx)
        const int64_t zlo = L - (I.nx - 1) - (I.ny - 1) > 0 ? L - (I.nx - 1) - (I.ny - 1) : 0;
        const int64_t zhi = L < I.nz - 1 ? L : I.nz - 1;
        const int64_t cnt = (zhi - zlo + 1) * I.ny;
        for (int64_t q = threadIdx.x; q < cnt && cnt > 0; q += blockDim.x) {
            const int64_t z = zlo + q / I.ny, y = q % I.ny, x = L - y - z;
            if (x >= 0 && x < I.nx) f(x, y, z, (z * I.ny + y) * I.nx + x);
        }
        (void)nyz;
        __syncthreads();
    }
}

// d: on entry diag(J) (nk_jacobian_diag), on exit D~
__global__ __launch_bounds__(1024) void k_ilu0_factor(IluArgs I, double* __restrict__ d) {
    ilu_levels(I, false, [&](int64_t x, int64_t y, int64_t z, int64_t i) {
        double a = d[i];
        if (z > 0) a = a - (I.cz / d[i - I.nx * I.ny]) * I.cz;
        if (y > 0) a = a - (I.cy / d[i - I.nx]) * I.cy;
        if (x > 0) a = a - (I.cx / d[i - 1]) * I.cx;
        d[i] = a;
    });
}

// z = U^-1 L^-1 v: forward sweep y_i = ((v_i - l_b y_b) - l_s y_s) - l_w y_w (into z), then the
// backward sweep z_i = (((y_i - c_x z_e) - c_y z_n) - c_z z_t) / D~_i
__global__ __launch_bounds__(1024) void k_ilu0_solve(IluArgs I, const double* __restrict__ d, double* __restrict__ zz,
                                                     const double* __restrict__ v) {
    ilu_levels(I, false, [&](int64_t x, int64_t y, int64_t z, int64_t i) {
        double a = v[i];
        if (z > 0) a = a - (I.cz / d[i - I.nx * I.ny]) * zz[i - I.nx * I.ny];
        if (y > 0) a = a - (I.cy / d[i - I.nx]) * zz[i - I.nx];
        if (x > 0) a = a - (I.cx / d[i - 1]) * zz[i - 1];
        zz[i] = a;
    });
    ilu_levels(I, true, [&](int64_t x, int64_t y, int64_t z, int64_t i) {
        double a = zz[i];
        if (x + 1 < I.nx) a = a - I.cx * zz[i + 1];
        if (y + 1 < I.ny) a = a - I.cy * zz[i + I.nx];
        if (z + 1 < I.nz) a = a - I.cz * zz[i + I.nx * I.ny];
        zz[i] = a / d[i];
    });
}

// ---- pipelined wavefront sweeps: one wave per 64-row strip, lanes skewed by one column --------
// Rows r = z ny + y of length nx (x fastest) are processed in order; point (x, r) needs (x - 1, r)
// (west: the lane's own previous step), (x, r - 1) (south: the lane above, one step earlier -- a
// shuffle; lane 0 reads the previous strip's last row) and (x, r - ny) (below: an earlier strip).
// At step t lane l handles column t - l, so a wave advances its 64 rows together, one column per
// step.  Strips hand over through per-strip progress counters (columns complete in every row):
// results are stored write-through (sc1), the wave drains its stores, then lane 0 publishes the
// counter (sc1); a consumer polls the counter (sc1) before its sc1 loads of those results
// (cdna_hip_programming.md §6 G16, the flag form).  Same arithmetic, in the same order per point, as
// the level sweep above and the oracle's loop: bit-identical.  The backward sweep is the forward
// one on reversed indices.  3D needs ny >= 64 (the plane below then lies in an earlier strip).
constexpr int kIluCh = 16;  // columns per chunk: loads issued together, progress checked / published once
struct IluPipe {
    IluArgs I;
    double* d;        // pivots (OP 0: diag(J) in, D~ out; else read-only)
    double* z;        // OP 1: y = L^-1 v out; OP 2: y in, z = U^-1 y out (in place)
    const double* v;  // OP 1: right-hand side
    int64_t* prog;    // per strip: leading columns complete in every row of the strip
    int* err;         // pinned host flag: a progress poll timed out
    int64_t R, S;     // rows (ny nz) and strips (ceil(R / 64))
    unsigned spin;    // polls per wave before giving up (~1 s)
};

__device__ __forceinline__ double ld_sc1(const double* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_sc1(double* p, double v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// wait until strip q has completed `need` leading columns (q < 0: nothing to wait for)
__device__ __forceinline__ bool ilu_wait(const IluPipe& P, int64_t q, int64_t need, unsigned& spins) {
    if (q < 0) return true;
    while (__hip_atomic_load(P.prog + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
        if (++spins > P.spin) {
            __hip_atomic_store(P.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    return true;
}

template <int OP>  // 0: factor D~ in place; 1: forward y = L^-1 v; 2: backward z = U^-1 y
__global__ __launch_bounds__(64) void k_ilu0_pipe(IluPipe P) {
    const int l = threadIdx.x;
    const int64_t nx = P.I.nx, ny = P.I.ny, nz = P.I.nz, nxny = nx * ny, R = P.R;
    const double cx = P.I.cx, cy = P.I.cy, cz = P.I.cz;
    // memory offsets of the processing-order neighbours (the backward sweep walks every axis reversed)
    const int64_t dS = OP == 2 ? nx : -nx, dB = OP == 2 ? nxny : -nxny;
    unsigned spins = 0;
    bool ok = true;
    for (int64_t s = blockIdx.x; s < P.S && ok; s += gridDim.x) {
        const int64_t rr = 64 * s + l;  // this lane's row in processing order
        const bool row_ok = rr < R;
        const int64_t r = OP == 2 ? R - 1 - rr : rr;
        const int64_t yy = row_ok ? r % ny : 0, zz = row_ok ? r / ny : 0;
        const bool has_s = row_ok && (OP == 2 ? yy + 1 < ny : yy > 0);
        const bool has_b = row_ok && (OP == 2 ? zz + 1 < nz : zz > 0);
        const int64_t last = (R - 1 - 64 * s) < 63 ? (R - 1 - 64 * s) : 63;  // last active lane
        // the earliest strip holding a "below" row of this strip (rows 64 s - ny ...); its successors
        // up to s - 1 have progressed at least as far (each strip waits for its predecessor)
        const int64_t sb = (nz > 1 && 64 * s - ny >= 0) ? (64 * s - ny) / 64 : -1;
        const int64_t sb2 = (nz > 1 && 64 * s + last - ny >= 0) ? (64 * s + last - ny) / 64 : -1;  // the last one
        const int64_t steps = nx + last;
        double prev = 0.0, prevd = 0.0;  // the lane's value (and OP 1: pivot) at its previous column
        for (int64_t t0 = 0; t0 < steps && ok; t0 += kIluCh) {
            const int64_t need = (t0 + kIluCh < nx) ? t0 + kIluCh : nx;
            ok = ilu_wait(P, s - 1, need, spins) && ilu_wait(P, sb, need, spins) &&
                 (sb2 == sb || sb2 == s - 1 || ilu_wait(P, sb2, need, spins));
            if (!ok) break;
            // every operand of the chunk's steps is independent of the recurrence: issue all loads
            // first (one memory round trip per chunk, not one per step), then run the chain
            // qa: own operand (D / v / y), qc: own pivot (OP 1, 2), qs: lane 0's south value (previous
            // strip), qb: south pivot (OP 1) or the below value (OP 0: pivot, OP 2: z), qd / qe: OP 1's
            // below pivot and below value
            double qa[kIluCh], qb[kIluCh], qc[kIluCh], qs[kIluCh], qd[kIluCh], qe[kIluCh];
#pragma unroll
            for (int k = 0; k < kIluCh; ++k) {
                const int64_t xp = t0 + k - l;
                const bool on = row_ok && xp >= 0 && xp < nx;
                const int64_t i = on ? r * nx + (OP == 2 ? nx - 1 - xp : xp) : 0;
                qa[k] = qb[k] = qc[k] = qs[k] = qd[k] = qe[k] = 0.0;
                if (on) {
                    if (l == 0 && has_s) qs[k] = ld_sc1((OP == 0 ? P.d : P.z) + i + dS);
                    if constexpr (OP == 0) {
                        qa[k] = P.d[i];
                        if (has_b) qb[k] = ld_sc1(P.d + i + dB);
                    } else if constexpr (OP == 1) {
                        qa[k] = P.v[i];
                        qc[k] = P.d[i];
                        if (has_s) qb[k] = P.d[i + dS];
                        if (has_b) {
                            qd[k] = P.d[i + dB];
                            qe[k] = ld_sc1(P.z + i + dB);
                        }
                    } else {
                        qa[k] = P.z[i];
                        qc[k] = P.d[i];
                        if (has_b) qb[k] = ld_sc1(P.z + i + dB);
                    }
                }
            }
            // OP 1: the L factors (c / pivot) do not depend on the recurrence: divide off the chain
            // (the same quotients, so the same rounding)
            double fb[kIluCh], fs[kIluCh], fw[kIluCh];
#pragma unroll
            for (int k = 0; k < kIluCh; ++k) {
                fb[k] = fs[k] = fw[k] = 0.0;
                if constexpr (OP == 1) {
                    const int64_t xp = t0 + k - l;
                    if (row_ok && xp >= 0 && xp < nx) {
                        if (has_b) fb[k] = cz / qd[k];
                        if (has_s) fs[k] = cy / qb[k];
                        if (xp > 0) fw[k] = cx / (k == 0 ? prevd : qc[k - 1]);
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < kIluCh; ++k) {
                const int64_t xp = t0 + k - l;
                const bool on = row_ok && xp >= 0 && xp < nx;
                const int64_t i = on ? r * nx + (OP == 2 ? nx - 1 - xp : xp) : 0;
                // south: lane l - 1's value of the previous step (same column, row rr - 1)
                double sv = __shfl_up(prev, 1, 64);
                if (l == 0) sv = qs[k];
                double a = 0.0, dcur = 0.0;
                if (on) {
                    if constexpr (OP == 0) {
                        a = qa[k];
                        if (has_b) a = a - (cz / qb[k]) * cz;
                        if (has_s) a = a - (cy / sv) * cy;
                        if (xp > 0) a = a - (cx / prev) * cx;
                    } else if constexpr (OP == 1) {
                        a = qa[k];
                        dcur = qc[k];
                        if (has_b) a = a - fb[k] * qe[k];
                        if (has_s) a = a - fs[k] * sv;
                        if (xp > 0) a = a - fw[k] * prev;
                    } else {
                        a = qa[k];
                        if (xp > 0) a = a - cx * prev;
                        if (has_s) a = a - cy * sv;
                        if (has_b) a = a - cz * qb[k];
                        a = a / qc[k];
                    }
                    st_sc1((OP == 0 ? P.d : P.z) + i, a);
                }
                prev = a;
                prevd = dcur;
            }
            // publish: every store of this chunk drained, then the strip's progress
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            int64_t done = t0 + kIluCh - last;
            done = done < 0 ? 0 : (done > nx ? nx : done);
            if (l == 0) __hip_atomic_store(P.prog + s, done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// off-diagonal entry of J along one axis: the exact tangent at point i of the unit vector on its
// neighbour (the entry collect(J) holds): lap = f / h^2 with f = 1 ((1 - α) for G_Midpoint!), the
// other axes add +0, Bratu adds λ (e^u · 0) = +0, heat: (Δt or Δt/2) (a lap) - 0
double ilu_offdiag(const nk_problem* p, double h) {
    const int sch = nk_is_heat(p->kind) ? nk_scheme(p->kind) : 0;
    const double f = sch == 1 ? (1.0 - p->alpha) * 1.0 : 1.0;
    const double lsum = ((f - 2.0 * 0.0) + 0.0) / (h * h);
    if (!nk_is_heat(p->kind)) return lsum;
    return (sch == 2 ? p->dt / 2.0 : p->dt) * (p->a * lsum) - 0.0;
}

IluArgs ilu_args(const nk_problem* p, int dim) {
    IluArgs I{};
    I.nx = p->nx; I.ny = p->ny; I.nz = p->nz;
    I.cx = ilu_offdiag(p, p->hx);
    I.cy = dim >= 2 ? ilu_offdiag(p, p->hy) : 0.0;
    I.cz = dim == 3 ? ilu_offdiag(p, p->hz) : 0.0;
    return I;
}

// the pipelined sweeps: rows of at least 64 columns... any 2D / 1D grid; 3D with ny >= 64 (the plane
// below a strip's rows must lie in an earlier strip); NK_ILU_PIPE=0 forces the level sweeps
static bool ilu_pipe_applies(nk_ctx* c, const nk_problem* p) {
    static const int pipe = NK_TUNE("NK_ILU_PIPE", 1);
    return pipe && c->ilu_pipe_ok && (p->nz == 1 || p->ny >= 64);
}

static int ilu_pipe_setup(nk_ctx* c, const nk_problem* p, int dim, IluPipe* P, int* grid) {
    P->I = ilu_args(p, dim);
    P->R = p->ny * p->nz;
    P->S = (P->R + 63) / 64;
    if (P->S > c->ilu_prog_cap) {
        if (c->ilu_prog) (void)hipFree(c->ilu_prog);
        c->ilu_prog = nullptr;
        c->ilu_prog_cap = 0;
        NK_HIP(c, hipMalloc(&c->ilu_prog, sizeof(int64_t) * (size_t)P->S));
        c->ilu_prog_cap = P->S;
    }
    if (!c->ilu_err) {
        NK_HIP(c, hipHostMalloc(&c->ilu_err, sizeof(int), hipHostMallocMapped));
        *c->ilu_err = 0;
        NK_HIP(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&c->ilu_err_dev), c->ilu_err, 0));
    }
    P->prog = c->ilu_prog;
    P->err = c->ilu_err_dev;
    P->spin = 1u << 22;  // polls before a strip gives up
    int dev = 0, cus = 0;
    NK_HIP(c, hipGetDevice(&dev));
    NK_HIP(c, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    // at most one wave per CU: every strip's predecessor is always running (no waiting wave can
    // keep it from being scheduled), and the sc1 hand-off stays in its measured form
    *grid = (int)std::min<int64_t>(P->S, std::max(1, cus));
    return NK_OK;
}

template <int OP>
static int ilu_pipe_launch(nk_ctx* c, const IluPipe& P, int grid, const char* name, double bytes) {
    NK_HIP(c, hipMemsetAsync(P.prog, 0, sizeof(int64_t) * (size_t)P.S, c->stream));
    return launch(c, name, bytes, [&] { hipLaunchKernelGGL(k_ilu0_pipe<OP>, dim3(grid), dim3(64), 0, c->stream, P); });
}

int launch_ilu0_factor(nk_ctx* c, const nk_problem* p, int dim, double* d) {
    const double bytes = 16.0 * (double)(p->nx * p->ny * p->nz);
    if (ilu_pipe_applies(c, p)) {
        IluPipe P{};
        int grid = 1;
        NK_TRY(ilu_pipe_setup(c, p, dim, &P, &grid));
        P.d = d;
        return ilu_pipe_launch<0>(c, P, grid, "ilu0_factor", bytes);
    }
    const IluArgs I = ilu_args(p, dim);
    return launch(c, "ilu0_factor_levels", bytes, [&] {
        hipLaunchKernelGGL(k_ilu0_factor, dim3(1), dim3(1024), 0, c->stream, I, d);
    });
}

// a pipelined sweep whose strip-progress poll timed out (ilu_err) left its output partial: wait for it,
// and if so turn the pipelined path off for this context and return 1 (the caller redoes the work on
// the one-work-group level sweep) -- the error never reaches a later call or a reused factor
int ilu_pipe_failed(nk_ctx* c) {
    if (!c->ilu_err) return 0;
    NK_HIP(c, hipStreamSynchronize(c->stream));
    if (!*(volatile int*)c->ilu_err) return 0;
    *c->ilu_err = 0;
    c->ilu_pipe_ok = false;
    std::fprintf(stderr, "[nkhip] pipelined ILU(0) sweep timed out; redone with the level sweep, which is used from now on\n");
    return 1;
}

int launch_ilu0_solve(nk_ctx* c, const nk_problem* p, int dim, const double* d, double* z, const double* v) {
    const double n = (double)(p->nx * p->ny * p->nz);
    if (ilu_pipe_applies(c, p)) {
        IluPipe P{};
        int grid = 1;
        NK_TRY(ilu_pipe_setup(c, p, dim, &P, &grid));
        P.d = const_cast<double*>(d);
        P.z = z;
        P.v = v;
        // the solve sweeps' poll limit (operational timeout): NK_ILU_SPIN_LIMIT shortens it for the
        // failure-path tests, which must see the solve sweeps -- not the factor -- time out
        static const unsigned spin = (unsigned)env_cfg("NK_ILU_SPIN_LIMIT", 1 << 22);
        P.spin = spin;
        // no host sync here (it would stall every Arnoldi step that applies the preconditioner): a
        // strip that timed out sets ilu_err, the next existing sync (mb_check) reports it, and the
        // Krylov solve / nk_precond_apply redoes its work once on the level sweep (ilu_redo)
        NK_TRY(ilu_pipe_launch<1>(c, P, grid, "ilu0_forward", 24.0 * n));  // v, d in; y out
        NK_TRY(ilu_pipe_launch<2>(c, P, grid, "ilu0_backward", 24.0 * n));  // y, d in; z out
        if (c->nranks == 1) return NK_OK;
        // Several ranks: the recovery must stay rank-local.  Redoing the whole Krylov solve on this rank
        // alone would re-enter reductions its peers have already moved past (the mailbox pairs them by
        // epoch): wrong scalars or a hang.  So check now (a host sync per apply, distributed ILU(0) only)
        // and redo this apply on the level sweep -- block Jacobi: the apply itself has no collective.
        const int bad = ilu_pipe_failed(c);
        if (bad <= 0) return bad;
    }
    const IluArgs I = ilu_args(p, dim);
    return launch(c, "ilu0_solve_levels", 48.0 * n, [&] {
        hipLaunchKernelGGL(k_ilu0_solve, dim3(1), dim3(1024), 0, c->stream, I, d, z, v);
    });
}

int launch_cg_direction(nk_ctx* c, int64_t n, double beta, double* p, const double* r) {
    NK_STREAM_LAUNCH("cg_direction", 24.0, k_cg_direction, n, beta, p, r);
}

// ------------------------------------------------------------------------------ variant bench hook
// Times kernel variants in ONE process (interleaved A/B, MI355X_MICROARCH methodology rule 24).
// Not part of the public ABI: exported as nkb_* by the kbench build only (tools/kbench*.py).
}  // namespace nk

#ifdef NK_KBENCH  // the nkb_* hooks: lib/libnkhip_kbench.so only (tools/, bench.py calibration)

// One Arnoldi step's MGS sweep at basis size k, as GMRES runs it: passes i = 1..k read q, V_i,
// V_{i+1} (the last one q, V_k) over a real basis of k+1 distinct vectors.  alt = alternate the
// sweep direction pass to pass.  Returns the average microseconds per pass.
extern "C" int nkb_mgs_seq(nk_ctx* c, int64_t n, int k, int variant, int alt, int reps, double* us_out) {
    using namespace nk;
    if (!c || n < 2 || k < 1 || reps < 1 || !us_out) return NK_E_ARG;
    std::vector<double*> V(k + 2, nullptr);
    for (size_t v = 0; v < V.size(); ++v) {  // non-zero data (zero-filled streams flatter HBM/DVFS)
        NK_HIP(c, hipMalloc(&V[v], sizeof(double) * n));
        NK_TRY(launch_fill(c, n, V[v], 0.37 + 0.01 * (double)v));
    }
    double* q = V[k + 1];
    const int g = red_blocks(n);
    double* parts[2] = {red_slot(c), red_slot(c)};  // ping-pong partials, as in the solver
    double* hs = c->scal;
    hipEvent_t a, b;
    NK_HIP(c, hipEventCreate(&a));
    NK_HIP(c, hipEventCreate(&b));
    auto sweep = [&] {
        for (int i = 0; i < k; ++i) {
            const int rev = alt ? (i & 1) : 0;
            const double* in = parts[i & 1];
            double* out = parts[(i + 1) & 1];
            if (i + 1 < k) mgs_dispatch<true>(variant, g, c->stream, n, q, V[i], V[i + 1], in, g, hs + 1, nullptr, out, rev, 0);
            else mgs_dispatch<false>(variant, g, c->stream, n, q, V[i], nullptr, in, g, hs + 1, nullptr, out, rev, 0);
        }
    };
    sweep();
    NK_HIP(c, hipEventRecord(a, c->stream));
    for (int r = 0; r < reps; ++r) sweep();
    NK_HIP(c, hipEventRecord(b, c->stream));
    NK_HIP(c, hipEventSynchronize(b));
    float ms = 0.f;
    NK_HIP(c, hipEventElapsedTime(&ms, a, b));
    *us_out = 1e3 * ms / ((double)reps * k);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    for (auto p : V) (void)hipFree(p);
    return NK_OK;
}

// 2D Bratu stencil variants: mode (0 res, 1 exact, 2 fd), epi, rows per tile, fast reciprocals.
extern "C" int nkb_stencil(nk_ctx* c, int64_t nx, int64_t ny, int mode, int epi, int rows, int fast, int reps,
                           double* us_out) {
    using namespace nk;
    if (!c || nx < 2 || ny < 2 || reps < 1 || !us_out) return NK_E_ARG;
    nk_problem p{NK_BRATU2D, NK_BC_ZERO, nx, ny, 1, 1.0 / (nx + 1), 1.0 / (ny + 1), 1.0, 3.51382, 0.0, 0.0, nullptr};
    double *u = nullptr, *v = nullptr, *F0 = nullptr, *aux = nullptr, *out = nullptr;
    for (double** q : {&u, &v, &F0, &aux, &out}) NK_TRY(nk_vec_alloc(c, &p, q));
    StencilIn in{&p, mode, epi, out, u, v, F0, aux, 1e-6};
    Red r{};
    hipEvent_t a, b;
    NK_HIP(c, hipEventCreate(&a));
    NK_HIP(c, hipEventCreate(&b));
    NK_TRY(launch_stencil_ex(c, in, &r, rows, fast));
    NK_HIP(c, hipEventRecord(a, c->stream));
    for (int k = 0; k < reps; ++k) NK_TRY(launch_stencil_ex(c, in, &r, rows, fast));
    NK_HIP(c, hipEventRecord(b, c->stream));
    NK_HIP(c, hipEventSynchronize(b));
    float ms = 0.f;
    NK_HIP(c, hipEventElapsedTime(&ms, a, b));
    *us_out = 1e3 * ms / reps;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    for (double* q : {u, v, F0, aux, out}) nk_vec_free(c, q);
    return NK_OK;
}

// 3D heat (implicit Euler) stencil variants at n^3: fast bits 8 / 16 select 8- / 16-row tiles
extern "C" int nkb_stencil3d(nk_ctx* c, int64_t n, int mode, int epi, int fast, int reps, double* us_out) {
    using namespace nk;
    if (!c || n < 2 || reps < 1 || !us_out) return NK_E_ARG;
    const double h = 1.0 / (n + 1);
    nk_problem p{NK_HEAT3D_EULER, NK_BC_ZERO, n, n, n, h, h, h, 0.0, 0.01, 1e-6, nullptr};
    double *u = nullptr, *v = nullptr, *F0 = nullptr, *aux = nullptr, *out = nullptr, *un = nullptr;
    p.un = reinterpret_cast<const double*>(1);  // geometry only while allocating
    for (double** q : {&u, &v, &F0, &aux, &out, &un}) NK_TRY(nk_vec_alloc(c, &p, q));
    p.un = un;
    StencilIn in{&p, mode, epi, out, u, v, F0, aux, 1e-6};
    Red r{};
    hipEvent_t a, b;
    NK_HIP(c, hipEventCreate(&a));
    NK_HIP(c, hipEventCreate(&b));
    NK_TRY(launch_stencil_ex(c, in, &r, 0, fast));
    NK_HIP(c, hipEventRecord(a, c->stream));
    for (int k = 0; k < reps; ++k) NK_TRY(launch_stencil_ex(c, in, &r, 0, fast));
    NK_HIP(c, hipEventRecord(b, c->stream));
    NK_HIP(c, hipEventSynchronize(b));
    float ms = 0.f;
    NK_HIP(c, hipEventElapsedTime(&ms, a, b));
    *us_out = 1e3 * ms / reps;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    for (double* q : {u, v, F0, aux, out, un}) nk_vec_free(c, q);
    return NK_OK;
}

// 3D heat stencil of `kind` (4 Euler / 6 midpoint / 8 trapezoid) at n x n x nz with `planes` per
// z-march (0: the launcher's choice) -- average microseconds per launch
extern "C" int nkb_stencil3d_ex(nk_ctx* c, int64_t n, int64_t nz, int kind, int mode, int epi, int planes, int fast,
                                int reps, double* us_out) {
    using namespace nk;
    if (!c || n < 3 || nz < 1 || reps < 1 || !us_out) return NK_E_ARG;
    const double h = 1.0 / (n + 1);
    nk_problem p{kind, NK_BC_ZERO, n, n, nz, h, h, h, 0.0, 0.01, 1e-6, nullptr, nullptr, 0.5};
    double *u = nullptr, *v = nullptr, *F0 = nullptr, *aux = nullptr, *out = nullptr, *un = nullptr;
    p.un = reinterpret_cast<const double*>(1);  // geometry only while allocating
    for (double** q : {&u, &v, &F0, &aux, &out, &un}) NK_TRY(nk_vec_alloc(c, &p, q));
    for (double* q : {u, v, F0, aux, un}) NK_TRY(launch_fill(c, n * n * nz, q, 0.25));
    p.un = un;
    StencilIn in{&p, mode, epi, out, u, v, F0, aux, 1e-6};
    Red r{};
    hipEvent_t a, b;
    NK_HIP(c, hipEventCreate(&a));
    NK_HIP(c, hipEventCreate(&b));
    NK_TRY(launch_stencil_ex(c, in, &r, planes, fast));
    NK_HIP(c, hipEventRecord(a, c->stream));
    for (int k = 0; k < reps; ++k) NK_TRY(launch_stencil_ex(c, in, &r, planes, fast));
    NK_HIP(c, hipEventRecord(b, c->stream));
    NK_HIP(c, hipEventSynchronize(b));
    float ms = 0.f;
    NK_HIP(c, hipEventElapsedTime(&ms, a, b));
    *us_out = 1e3 * ms / reps;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    for (double* q : {u, v, F0, aux, out, un}) nk_vec_free(c, q);
    return NK_OK;
}

// any stencil kind at nx x ny x nz (nz = 1 for the 2D kinds): mode / epi, rows (2D: rows per tile;
// 3D: planes per z-march; 0: the launcher's choice), variant bits `fast` -- microseconds per launch
extern "C" int nkb_stencil_kind(nk_ctx* c, int kind, int64_t nx, int64_t ny, int64_t nz, int mode, int epi, int rows,
                                int fast, int reps, double* us_out) {
    using namespace nk;
    if (!c || nx < 3 || ny < 3 || nz < 1 || reps < 1 || !us_out || kind < NK_BRATU2D || kind > NK_HEAT3D_TRAPEZOID)
        return NK_E_ARG;
    const double h = 1.0 / (nx + 1);
    // hook-only bits: 128 bc_periodic!, 256 the fused normalisation (v / h stored as V_k: the Arnoldi Jv)
    const bool per = (fast & 128) != 0, vfuse = (fast & 256) != 0;
    fast &= ~(128 | 256);
    nk_problem p{kind, per ? NK_BC_PERIODIC : NK_BC_ZERO, nx, ny, nz, h, h, h, 3.51382, 0.01, 1e-6, nullptr, nullptr, 0.5};
    double *u = nullptr, *v = nullptr, *F0 = nullptr, *aux = nullptr, *out = nullptr, *un = nullptr, *vk = nullptr;
    p.un = reinterpret_cast<const double*>(1);  // geometry only while allocating
    for (double** q : {&u, &v, &F0, &aux, &out, &un, &vk}) NK_TRY(nk_vec_alloc(c, &p, q));
    for (double* q : {u, v, F0, aux, un}) NK_TRY(launch_fill(c, nx * ny * nz, q, 0.25));
    p.un = un;
    StencilIn in{&p, mode, epi, out, u, v, F0, aux, 1e-6};
    in.f0r = (fast & 32) != 0;  // variant bit 32: F0 recomputed (the F0R kernels, where the policy allows)
    if (vfuse && mode != MODE_RES && epi == EPI_DOT) {
        NK_TRY(launch_fill(c, 1, c->scal + 32, 2.0));
        in.vdiv = c->scal + 32;
        in.vout = vk;
    }
    Red r{};
    hipEvent_t a, b;
    NK_HIP(c, hipEventCreate(&a));
    NK_HIP(c, hipEventCreate(&b));
    NK_TRY(launch_stencil_ex(c, in, &r, rows, fast));
    NK_HIP(c, hipEventRecord(a, c->stream));
    for (int k = 0; k < reps; ++k) NK_TRY(launch_stencil_ex(c, in, &r, rows, fast));
    NK_HIP(c, hipEventRecord(b, c->stream));
    NK_HIP(c, hipEventSynchronize(b));
    float ms = 0.f;
    NK_HIP(c, hipEventElapsedTime(&ms, a, b));
    *us_out = 1e3 * ms / reps;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    for (double* q : {u, v, F0, aux, out, un, vk}) nk_vec_free(c, q);
    return NK_OK;
}

// Two stencil variants (fast bits fa / fb, incl. the hook-only bits 128 periodic / 256 fused
// normalisation) on the same pseudo-random operands: diff[0] = max |out_a - out_b|, diff[1] = the same
// for the stored V_k, diff[2] / diff[3] = the two reductions' sums (epi != none), diff[4] = max |out_a|
namespace nk {
namespace {
__global__ __launch_bounds__(kBlock) void k_hashfill2(int64_t n, double* __restrict__ x, uint64_t seed, double lo, double hi) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        uint64_t z = (uint64_t)i * 0x9e3779b97f4a7c15ull + seed;
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        z ^= z >> 31;
        x[i] = lo + (hi - lo) * ((double)(z >> 11) * 0x1.0p-53);
    }
}
}  // namespace
}  // namespace nk

extern "C" int nkb_stencil_cmp(nk_ctx* c, int kind, int64_t nx, int64_t ny, int64_t nz, int mode, int epi, int fa, int fb,
                               double* diff) {
    using namespace nk;
    if (!c || nx < 3 || ny < 3 || nz < 1 || !diff || kind < NK_BRATU2D || kind > NK_HEAT3D_TRAPEZOID) return NK_E_ARG;
    const double h = 1.0 / (nx + 1);
    const bool per = (fa & 128) != 0, vfuse = (fa & 256) != 0;
    nk_problem p{kind, per ? NK_BC_PERIODIC : NK_BC_ZERO, nx, ny, nz, h, h, h, 3.51382, 0.01, 1e-6, nullptr, nullptr, 0.3};
    double *u = nullptr, *v = nullptr, *F0 = nullptr, *aux = nullptr, *un = nullptr, *oa = nullptr, *ob = nullptr,
           *va = nullptr, *vb = nullptr;
    p.un = reinterpret_cast<const double*>(1);
    for (double** q : {&u, &v, &F0, &aux, &un, &oa, &ob, &va, &vb}) NK_TRY(nk_vec_alloc(c, &p, q));
    const int64_t n = nx * ny * nz;
    uint64_t seed = 17;
    for (double* q : {u, v, F0, aux, un}) {
        hipLaunchKernelGGL(k_hashfill2, dim3(2048), dim3(kBlock), 0, c->stream, n, q, seed, -1.0, 1.0);
        seed += 7919;
    }
    p.un = un;
    NK_TRY(launch_fill(c, 1, c->scal + 32, 1.7));
    // F0 as the residual kernel computes it (the F0R kernels rely on it)
    {
        StencilIn r{&p, MODE_RES, EPI_NONE, F0, u, nullptr, nullptr, nullptr, 0.0};
        Red rr{};
        NK_TRY(launch_stencil_ex(c, r, &rr, 0, 0));
    }
    double sums[2] = {0.0, 0.0};
    for (int which = 0; which < 2; ++which) {
        int f = which ? fb : fa;
        f &= ~(128 | 256);
        StencilIn in{&p, mode, epi, which ? ob : oa, u, v, F0, aux, 1e-6};
        in.f0r = (f & 32) != 0;
        if (vfuse && mode != MODE_RES && epi == EPI_DOT) {
            in.vdiv = c->scal + 32;
            in.vout = which ? vb : va;
        }
        Red r{};
        NK_TRY(launch_stencil_ex(c, in, &r, 0, f));
        if (epi != EPI_NONE) {
            NK_TRY(launch_finalize(c, r, c->scal + 40 + which, 0, nullptr));
        }
    }
    NK_HIP(c, hipStreamSynchronize(c->stream));
    if (epi != EPI_NONE) NK_HIP(c, hipMemcpy(sums, c->scal + 40, 2 * sizeof(double), hipMemcpyDeviceToHost));
    std::vector<double> a(n), b(n);
    double d0 = 0.0, d1 = 0.0, m = 0.0;
    NK_HIP(c, hipMemcpy(a.data(), oa, sizeof(double) * n, hipMemcpyDeviceToHost));
    NK_HIP(c, hipMemcpy(b.data(), ob, sizeof(double) * n, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < n; ++i) {
        d0 = std::max(d0, std::fabs(a[i] - b[i]));
        m = std::max(m, std::fabs(a[i]));
    }
    if (vfuse) {
        NK_HIP(c, hipMemcpy(a.data(), va, sizeof(double) * n, hipMemcpyDeviceToHost));
        NK_HIP(c, hipMemcpy(b.data(), vb, sizeof(double) * n, hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < n; ++i) d1 = std::max(d1, std::fabs(a[i] - b[i]));
    }
    diff[0] = d0;
    diff[1] = d1;
    diff[2] = sums[0];
    diff[3] = sums[1];
    diff[4] = m;
    for (double* q : {u, v, F0, aux, un, oa, ob, va, vb}) nk_vec_free(c, q);
    return NK_OK;
}

// x update of a GMRES cycle with k basis vectors (xr = 0 start, Newton update fused into u, ||u||
// partials), with U elements per thread (NK_UPD_U) -- average microseconds per launch
extern "C" int nkb_update_x(nk_ctx* c, int64_t n, int k, int u_elems, int reps, double* us_out) {
    using namespace nk;
    if (!c || n < 2 || k < 1 || k > kMaxUpdateVecs || reps < 1 || !us_out) return NK_E_ARG;
    std::vector<double*> V(k + 3, nullptr);
    for (size_t v = 0; v < V.size(); ++v) {
        NK_HIP(c, hipMalloc(&V[v], sizeof(double) * n));
        NK_TRY(launch_fill(c, n, V[v], 0.37 + 0.01 * (double)v));
    }
    double *x = V[k], *xr = V[k + 1], *u = V[k + 2];
    double* y = c->scal + 16;
    std::vector<double> yh(k, 1e-3);
    NK_HIP(c, hipMemcpy(y, yh.data(), sizeof(double) * k, hipMemcpyHostToDevice));
    const int g = red_blocks(n);
    UpdArgs A{};
    for (int i = 0; i < k; ++i) A.V[i] = V[i];
    A.x = x; A.xr = xr; A.y = y; A.n = n; A.k = k; A.first = 1; A.last = 1; A.restart = 0; A.u = u;
    A.part = red_slot(c);
    A.fin = 0;
    auto go = [&] {
        if (u_elems >= 8) hipLaunchKernelGGL(k_update_x<8>, dim3(g), dim3(kBlock), 0, c->stream, A);
        else if (u_elems >= 4) hipLaunchKernelGGL(k_update_x<4>, dim3(g), dim3(kBlock), 0, c->stream, A);
        else if (u_elems == 2) hipLaunchKernelGGL(k_update_x<2>, dim3(g), dim3(kBlock), 0, c->stream, A);
        else hipLaunchKernelGGL(k_update_x<1>, dim3(g), dim3(kBlock), 0, c->stream, A);
    };
    hipEvent_t a, b;
    NK_HIP(c, hipEventCreate(&a));
    NK_HIP(c, hipEventCreate(&b));
    go();
    NK_HIP(c, hipEventRecord(a, c->stream));
    for (int r = 0; r < reps; ++r) go();
    NK_HIP(c, hipEventRecord(b, c->stream));
    NK_HIP(c, hipEventSynchronize(b));
    float ms = 0.f;
    NK_HIP(c, hipEventElapsedTime(&ms, a, b));
    *us_out = 1e3 * ms / reps;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    for (double* v : V) (void)hipFree(v);
    return NK_OK;
}

// The achievable-bandwidth calibration point: the fastest plain copy the stream probe found
// (tools/stream_probe.py, profiles/r02/stream_probe.log): one 16-B element per thread, one block
// per 256 elements, non-temporal load and store -- 6.2-6.5 TB/s, against 5.0 for a grid of 8
// blocks per CU looping over block chunks (the calibration of the earlier round-2 bench lines).
namespace nk {
namespace {
__global__ __launch_bounds__(kBlock) void k_copy_cal(int64_t n2, dx2* __restrict__ y, const dx2* __restrict__ x) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n2) __builtin_nontemporal_store(__builtin_nontemporal_load(x + i), y + i);
}
}  // namespace
}  // namespace nk

extern "C" int nkb_copy(nk_ctx* c, int64_t n, int reps, double* us_out) {
    using namespace nk;
    if (!c || n < 2 || reps < 1 || !us_out) return NK_E_ARG;
    double *x = nullptr, *y = nullptr;
    NK_HIP(c, hipMalloc(&x, sizeof(double) * n));
    // NK_ALLOC_STAGGER=<bytes>: y starts that far into its allocation (the vector start-offset probe, §3)
    const size_t ys = (size_t)std::max(0, NK_TUNE("NK_ALLOC_STAGGER", 0)) / 256 * 32;
    NK_HIP(c, hipMalloc(&y, sizeof(double) * (n + ys)));
    double* const ybase = y;
    y += ys;
    NK_HIP(c, hipMemsetAsync(x, 0, sizeof(double) * n, c->stream));
    hipEvent_t a, b;
    NK_HIP(c, hipEventCreate(&a));
    NK_HIP(c, hipEventCreate(&b));
    const int64_t n2 = n / 2;  // the calibration counts 16 B per element pair moved: n even
    const int64_t g = (n2 + kBlock - 1) / kBlock;
    if (g > INT32_MAX) return NK_E_ARG;
    auto go = [&] {
        hipLaunchKernelGGL(k_copy_cal, dim3((unsigned)g), dim3(kBlock), 0, c->stream, n2, reinterpret_cast<dx2*>(y),
                           reinterpret_cast<const dx2*>(x));
    };
    go();
    NK_HIP(c, hipEventRecord(a, c->stream));
    for (int r = 0; r < reps; ++r) go();
    NK_HIP(c, hipEventRecord(b, c->stream));
    NK_HIP(c, hipEventSynchronize(b));
    float ms = 0.f;
    NK_HIP(c, hipEventElapsedTime(&ms, a, b));
    *us_out = 1e3 * ms / reps;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    (void)hipFree(x);
    (void)hipFree(ybase);
    return NK_OK;
}

// ------------------------------------------------------------------------------ streaming probe
// HBM streaming-rate probe behind tools/stream_probe.py: copy y = x (R = 1) or the MGS access
// pattern q -= s v; <w, q> (R = 3 reads + 1 write) with U 16-B loads per stream in flight per
// thread, in one of three orders: ORD 0 grid-stride (the U loads one grid apart), ORD 1 block-
// contiguous chunks, ORD 2 grid-stride with each block's U loads on consecutive 4 KB pieces.
namespace nk {
namespace {
template <int U, int ORD, int R, bool NTL, bool NTS = false>
__global__ __launch_bounds__(kBlock) void k_stream_probe(int64_t n2, dx2* __restrict__ q, const dx2* __restrict__ v,
                                                        const dx2* __restrict__ w, double* __restrict__ part) {
    const int64_t nthr = (int64_t)gridDim.x * kBlock;
    int64_t i, st, ust, end;
    if constexpr (ORD == 1) {
        const int64_t per = (n2 + gridDim.x - 1) / gridDim.x;
        i = (int64_t)blockIdx.x * per + threadIdx.x;
        end = (int64_t)(blockIdx.x + 1) * per < n2 ? (int64_t)(blockIdx.x + 1) * per : n2;
        st = kBlock;
        ust = (int64_t)U * kBlock;
    } else if constexpr (ORD == 2) {
        i = (int64_t)blockIdx.x * kBlock * U + threadIdx.x;
        end = n2;
        st = kBlock;
        ust = nthr * U;
    } else {
        i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
        end = n2;
        st = nthr;
        ust = nthr * U;
    }
    double acc = 0.0;
    for (; i + (U - 1) * st < end; i += ust) {
        dx2 a[U], b[U], c[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (R == 1) {
                a[u] = ld2<NTL>(v + i + u * st);
            } else {
                a[u] = ld2<false>(q + i + u * st);
                b[u] = ld2<NTL>(v + i + u * st);
                c[u] = ld2<false>(w + i + u * st);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (R == 3) {
                a[u].x = fma(-0.5, b[u].x, a[u].x);
                a[u].y = fma(-0.5, b[u].y, a[u].y);
                acc = fma(c[u].x, a[u].x, acc);
                acc = fma(c[u].y, a[u].y, acc);
            }
            st2<NTS>(q + i + u * st, a[u]);
        }
    }
    if (acc == 12345.0) part[0] = acc;  // keeps the dot live
}
}  // namespace
}  // namespace nk

extern "C" int nkb_stream(nk_ctx* c, int64_t n, int variant, int grid, int reps, double* us_out) {
    using namespace nk;
    if (!c || n < 2 || reps < 1 || !us_out) return NK_E_ARG;
    double *q = nullptr, *v = nullptr, *w = nullptr;
    NK_HIP(c, hipMalloc(&q, sizeof(double) * n));
    NK_HIP(c, hipMalloc(&v, sizeof(double) * n));
    NK_HIP(c, hipMalloc(&w, sizeof(double) * n));
    NK_TRY(launch_fill(c, n, q, 1.0));
    NK_TRY(launch_fill(c, n, v, 1e-3));
    NK_TRY(launch_fill(c, n, w, 2.0));
    const int g = grid > 0 ? grid : red_blocks(n);
    const int64_t n2 = n / 2;
    dx2* qs = reinterpret_cast<dx2*>(q);
    const dx2* vs = reinterpret_cast<const dx2*>(v);
    const dx2* ws = reinterpret_cast<const dx2*>(w);
    double* part = red_slot(c);
#define NKB_S(U, O, R, NT) hipLaunchKernelGGL((k_stream_probe<U, O, R, NT>), dim3(g), dim3(kBlock), 0, c->stream, n2, qs, vs, ws, part)
#define NKB_SN(U, O, NL) hipLaunchKernelGGL((k_stream_probe<U, O, 1, NL, true>), dim3(g), dim3(kBlock), 0, c->stream, n2, qs, vs, ws, part)
    auto go = [&] {
        switch (variant) {  // R=1: y(q) = x(v)    R=3: MGS pattern
        case 0: NKB_S(1, 0, 1, false); break;
        case 1: NKB_S(2, 0, 1, false); break;
        case 2: NKB_S(4, 0, 1, false); break;
        case 3: NKB_S(2, 1, 1, false); break;
        case 4: NKB_S(4, 1, 1, false); break;
        case 5: NKB_S(2, 2, 1, false); break;
        case 6: NKB_S(4, 2, 1, false); break;
        case 7: NKB_S(1, 0, 3, true); break;
        case 8: NKB_S(2, 0, 3, true); break;
        case 9: NKB_S(2, 1, 3, true); break;
        case 10: NKB_S(4, 1, 3, true); break;
        case 11: NKB_S(2, 2, 3, true); break;
        case 12: NKB_S(4, 2, 3, true); break;
        case 14: NKB_S(1, 0, 1, true); break;    // copy, non-temporal load
        case 15: NKB_SN(1, 0, true); break;      // copy, non-temporal load and store
        case 16: NKB_SN(1, 0, false); break;     // copy, non-temporal store
        case 17: NKB_SN(4, 1, true); break;      // copy U4 chunk, non-temporal load and store
        case 18: NKB_SN(2, 0, true); break;      // copy U2 grid-stride, non-temporal load and store
        default: NKB_S(1, 1, 3, true); break;
        }
    };
#undef NKB_S
#undef NKB_SN
    hipEvent_t a, b;
    NK_HIP(c, hipEventCreate(&a));
    NK_HIP(c, hipEventCreate(&b));
    go();
    NK_HIP(c, hipEventRecord(a, c->stream));
    for (int r = 0; r < reps; ++r) go();
    NK_HIP(c, hipEventRecord(b, c->stream));
    NK_HIP(c, hipEventSynchronize(b));
    float ms = 0.f;
    NK_HIP(c, hipEventElapsedTime(&ms, a, b));
    *us_out = 1e3 * ms / reps;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    (void)hipFree(q);
    (void)hipFree(v);
    (void)hipFree(w);
    return NK_OK;
}

// The FD Jv's stream pattern without its arithmetic (the 2D march's floor): four reads (u, v,
// F0, V_1) and one write per point, a dot kept live -- what the memory system gives 4R + 1W at all,
// against the copy's 1R + 1W.  ORD 0 grid-stride, 1 block-contiguous chunks; U 16-B loads per stream.
namespace nk {
namespace {
template <int U, int ORD>
__global__ __launch_bounds__(kBlock) void k_stream_jv(int64_t n2, dx2* __restrict__ out, const dx2* __restrict__ a,
                                                     const dx2* __restrict__ b, const dx2* __restrict__ f,
                                                     const dx2* __restrict__ w, double* __restrict__ part) {
    const int64_t nthr = (int64_t)gridDim.x * kBlock;
    int64_t i, st, ust, end;
    if constexpr (ORD == 1) {
        const int64_t per = (n2 + gridDim.x - 1) / gridDim.x;
        i = (int64_t)blockIdx.x * per + threadIdx.x;
        end = (int64_t)(blockIdx.x + 1) * per < n2 ? (int64_t)(blockIdx.x + 1) * per : n2;
        st = kBlock;
        ust = (int64_t)U * kBlock;
    } else {
        i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
        end = n2;
        st = nthr;
        ust = nthr * U;
    }
    double acc = 0.0;
    for (; i + (U - 1) * st < end; i += ust) {
        dx2 x[U], y[U], z[U], t[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            x[u] = ld2<false>(a + i + u * st);
            y[u] = ld2<false>(b + i + u * st);
            z[u] = ld2<false>(f + i + u * st);
            t[u] = ld2<false>(w + i + u * st);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            dx2 r;
            r.x = fma(1e-7, y[u].x, x[u].x) - z[u].x;
            r.y = fma(1e-7, y[u].y, x[u].y) - z[u].y;
            acc = fma(t[u].x, r.x, acc);
            acc = fma(t[u].y, r.y, acc);
            st2<false>(out + i + u * st, r);
        }
    }
    for (; i < end; i += st) {  // the remainder (fewer than U strides left)
        const dx2 x = ld2<false>(a + i), y = ld2<false>(b + i), z = ld2<false>(f + i), t = ld2<false>(w + i);
        dx2 r;
        r.x = fma(1e-7, y.x, x.x) - z.x;
        r.y = fma(1e-7, y.y, x.y) - z.y;
        acc = fma(t.x, r.x, acc);
        acc = fma(t.y, r.y, acc);
        st2<false>(out + i, r);
    }
    if (acc == 12345.0) part[0] = acc;  // keeps the dot live
}
}  // namespace
}  // namespace nk

extern "C" int nkb_stream_jv(nk_ctx* c, int64_t n, int variant, int grid, int reps, double* us_out) {
    using namespace nk;
    if (!c || n < 2 || reps < 1 || !us_out) return NK_E_ARG;
    double* buf[5] = {};
    for (auto& x : buf) {
        NK_HIP(c, hipMalloc(&x, sizeof(double) * n));
        NK_TRY(launch_fill(c, n, x, 1.0));
    }
    const int g = grid > 0 ? grid : red_blocks(n);
    const int64_t n2 = n / 2;
    auto d = [&](int k) { return reinterpret_cast<dx2*>(buf[k]); };
    double* part = red_slot(c);
    auto go = [&] {
        switch (variant) {
        case 0: hipLaunchKernelGGL((k_stream_jv<1, 0>), dim3(g), dim3(kBlock), 0, c->stream, n2, d(0), d(1), d(2), d(3), d(4), part); break;
        case 1: hipLaunchKernelGGL((k_stream_jv<2, 0>), dim3(g), dim3(kBlock), 0, c->stream, n2, d(0), d(1), d(2), d(3), d(4), part); break;
        case 2: hipLaunchKernelGGL((k_stream_jv<2, 1>), dim3(g), dim3(kBlock), 0, c->stream, n2, d(0), d(1), d(2), d(3), d(4), part); break;
        default: hipLaunchKernelGGL((k_stream_jv<4, 1>), dim3(g), dim3(kBlock), 0, c->stream, n2, d(0), d(1), d(2), d(3), d(4), part); break;
        }
    };
    hipEvent_t a, b;
    NK_HIP(c, hipEventCreate(&a));
    NK_HIP(c, hipEventCreate(&b));
    go();
    NK_HIP(c, hipEventRecord(a, c->stream));
    for (int r = 0; r < reps; ++r) go();
    NK_HIP(c, hipEventRecord(b, c->stream));
    NK_HIP(c, hipEventSynchronize(b));
    float ms = 0.f;
    NK_HIP(c, hipEventElapsedTime(&ms, a, b));
    *us_out = 1e3 * ms / reps;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    for (auto x : buf) (void)hipFree(x);
    return NK_OK;
}
#endif  // NK_KBENCH
