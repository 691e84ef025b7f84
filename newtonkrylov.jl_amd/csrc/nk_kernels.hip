// nk_kernels.hip -- the hand-written gfx950 kernels of the JFNK inner loop and their launchers: BLAS-1,
// the per-pass MGS chain, the x update, the stencil dispatch (launch_stencil_ex), NK_USER pieces.
// Ghost planes / faces / the peer mailbox: nk_halo.hip; CG, Jacobi, ILU(0): nk_precond.hip; the
// kernel-variant bench hooks: nk_kbench.hip (and the two here that need this unit's templates).
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
// NT marks the loads/stores non-temporal (streams that are not re-read soon; ld2 / st2, nk_device.hpp).
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

}  // namespace

// this unit's copy of the mailbox binding (mailbox_bind, nk_halo.hip, sets every unit's)
hipError_t kernels_bind_mb(const MbInfo& m) { return hipMemcpyToSymbol(HIP_SYMBOL(g_mb), &m, sizeof(m)); }

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
// 3D blocks: may a Jv launch carry its ghost layers itself (blk_tile_exchange)?  Every rank must decide alike
// (tile flags vs k_faces_ipc's block flags), so from values every rank holds alike: the largest block of the
// grid from the global spacings (one rank: its own), the most ranks on one GPU.  Each face's patches need a
// flag each; a z-partner pair sits tiles_x x tiles_y dispatch positions apart, which must stay within one
// tile per CU so that every waiting tile's partner is resident; ranks sharing a GPU only for small blocks.
bool blk_inlaunch_ok(nk_ctx* c, const nk_problem* p, int64_t fuse_max) {
    int64_t bx = p->nx, by = p->ny, bz = p->nz;
    if (c->nranks > 1) {
        auto glob = [](double h) { return (h > 0.0 && 1.0 / h < 1e15) ? std::max<int64_t>(1, std::llround(1.0 / h) - 1) : -1; };
        const int64_t NX = glob(p->hx), NY = glob(p->hy), NZ = glob(p->hz);
        const int pz = c->nranks / (c->px * c->py);
        if (NX < 0 || NY < 0 || NZ < 0) return false;
        bx = (NX + c->px - 1) / c->px;
        by = (NY + c->py - 1) / c->py;
        bz = (NZ + pz - 1) / pz;
    }
    if (!c->n_cus && (hipDeviceGetAttribute(&c->n_cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || c->n_cus < 1)) {
        (void)hipGetLastError();
        c->n_cus = 0;
        return false;
    }
    const int64_t vec = bx % 2 == 0 ? 2 : 1;
    const int64_t tx = (bx + 64 * vec - 1) / (64 * vec), ty = (by + 3) / 4, nzc = (bz + 15) / 16;
    if (tx * ty > kHaloTileFlags || tx * nzc > kHaloTileFlags || ty * nzc > kHaloTileFlags) return false;
    if (tx * ty > c->n_cus) return false;
    if (std::max({bx * by, bx * bz, by * bz}) > c->halo_cap) return false;
    return c->share_most <= 1 || bx * by * bz <= fuse_max;
}

// the dispatch order of an in-launch block exchange: the exchanging tiles first, in pair order -- z-chunks
// 0, last, 1, last - 1, ..., rows of tiles likewise, columns innermost -- so each tile's x / y / z partner
// is at most 1 / tiles_x / tiles_x tiles_y positions away; then the other tiles in XCD bands (plane-major)
int blk_order(nk_ctx* c, const KArgs& A, int nzc, const int** out) {
    const int tx_n = A.tiles_x, ty_n = A.tiles_y, tpl = tx_n * ty_n, n = tpl * nzc;
    int mask = 0;
    for (int s = 0; s < kHaloSides; ++s) mask |= (A.bnbr[s] >= 0) << s;
    const uint64_t key = ((uint64_t)tx_n << 44) ^ ((uint64_t)ty_n << 24) ^ ((uint64_t)nzc << 6) ^ (uint64_t)mask;
    if (c->blk_order && c->blk_order_key == key) {
        *out = c->blk_order;
        return NK_OK;
    }
    auto ord = [](int i, int m) { return (i & 1) ? m - 1 - (i >> 1) : (i >> 1); };
    auto exch = [&](int tz, int ty, int tx) {
        return ((mask & 1) && tz == 0) || ((mask & 2) && tz == nzc - 1) || ((mask & 4) && ty == 0) ||
               ((mask & 8) && ty == ty_n - 1) || ((mask & 16) && tx == 0) || ((mask & 32) && tx == tx_n - 1);
    };
    std::vector<int> order, rest;
    order.reserve(n);
    std::vector<char> seen((size_t)n, 0);
    for (int zi = 0; zi < nzc; ++zi)
        for (int yi = 0; yi < ty_n; ++yi)
            for (int tx = 0; tx < tx_n; ++tx) {
                const int tz = ord(zi, nzc), ty = ord(yi, ty_n);
                if (exch(tz, ty, tx)) {
                    order.push_back(tz * tpl + ty * tx_n + tx);
                    seen[(size_t)(tz * tpl + ty * tx_n + tx)] = 1;
                }
            }
    for (int t = 0; t < n; ++t)
        if (!seen[(size_t)t]) rest.push_back(t);
    const int m = (int)rest.size(), m8 = m & ~7;
    for (int i = 0; i < m; ++i)  // block i of the rest lands on XCD i % 8 and takes that XCD's band's (i / 8)-th tile
        order.push_back(rest[(size_t)(i < m8 ? (i & 7) * (m8 >> 3) + (i >> 3) : i)]);
    if (c->blk_order_cap < n) {
        if (c->blk_order) (void)hipFree(c->blk_order);
        c->blk_order = nullptr;
        c->blk_order_cap = 0;
        NK_HIP(c, hipMalloc(reinterpret_cast<void**>(&c->blk_order), sizeof(int) * (size_t)n));
        c->blk_order_cap = n;
    }
    NK_HIP(c, hipMemcpyAsync(c->blk_order, order.data(), sizeof(int) * (size_t)n, hipMemcpyHostToDevice, c->stream));
    NK_HIP(c, hipStreamSynchronize(c->stream));  // (the host vector goes out of scope; once per geometry)
    c->blk_order_key = key;
    *out = c->blk_order;
    return NK_OK;
}
}  // namespace

int launch_stencil(nk_ctx* c, const StencilIn& in, Red* red) {
    if (in.p && nk_is_user(in.p->kind)) {
        if (in.xchg_v) NK_TRY(halo_exchange(c, in.p, in.v));
        return launch_user(c, in, red);
    }
    return launch_stencil_ex(c, in, red, 0, 0);
}


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
        if (planes < min_planes || A.blk) planes = min_planes;  // (blocks: one chunk size on every rank -- the
                                                                 //  in-launch exchange numbers x / y patches by chunk)
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
        // on CUs the peer's producing tiles need (r05: 8 ranks x 256^2 x 32 planes, 30.5 s per step fused;
        // 26.7 ms with the exchange kernel, profiles/r06/rehearsal8_heat3d_256_slabs.json, the default
        // spin limit).  Neighbours must agree on the form (tile flags vs
        // the exchange kernel's block flags), so the test uses rank-uniform values only: the most ranks on
        // one GPU and the slab size estimated from the global spacing, never this rank's slab
        static const int64_t fuse_max = env_cfg("NK_SHARED_FUSE_MAX", 0) > 0 ? env_cfg("NK_SHARED_FUSE_MAX", 0) : kSharedFuseMax;
        const bool share_ok = c->share_most <= 1 || shared_slab_points(c, p, g) <= fuse_max;
        const bool fuse = fuse_env && c->mb_on && (c->nranks > 1 || self) && share_ok && !per && !A.blk && in.mode != MODE_RES &&
                          (g.dim == 2 || (g.dim == 3 && A.lds3)) && g.plane <= c->halo_cap && tiles_pl <= kHaloTileFlags;
        if (A.blk) {  // 3D blocks: k_faces_ipc first, or (opt-in) every ghost layer inside this launch
            // In-launch (blk_tile_exchange) is bitwise the same but SLOWER on one GPU, the only place it can be
            // measured here: the self-block 256^3 Jv 145 + 22 us (faces kernel) -> 187 us in-launch (2x2x2, every
            // tile exchanges x patches and waits a round trip), 145 + 21 -> 172 us at 1x2x4 (profiles/r06/
            // ab_blk_*.json).  NK_BLK_INLAUNCH=1 keeps it reachable for xGMI, where the separate kernel's
            // transfer -- not a round trip -- would dominate (unmeasured)
            static const int blk_in_env = env_cfg("NK_BLK_INLAUNCH", 0);
            const bool bfuse = blk_in_env && fuse_env && c->mb_on && in.mode != MODE_RES && rows_override <= 0 &&
                               blk_inlaunch_ok(c, p, fuse_max);
            if (bfuse) {
                ++c->n_jv_halo_fused;
                A.hx_blk = 1;
                A.hx_epoch = ++c->halo_epoch;
                A.hx_cap = c->halo_cap;
                for (int sd = 0; sd < kHaloSides; ++sd) A.bnbr[sd] = block_nbr(c, sd);
                NK_TRY(blk_order(c, A, (int)((p->nz + A.rows - 1) / A.rows), &A.torder));
            } else {
                ++c->n_jv_halo_separate;
                NK_TRY(halo_exchange(c, p, in.v));
            }
        } else if (fuse) {
            ++c->n_jv_halo_fused;
            A.hx_lo = c->rank > 0 || self;
            A.hx_hi = c->rank + 1 < c->nranks || self;
            A.hx_epoch = ++c->halo_epoch;
            A.hx_cap = c->halo_cap;
        } else {
            if (c->nranks > 1 || per || self || block_self(c)) ++c->n_jv_halo_separate;
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
#endif  // NK_KBENCH
