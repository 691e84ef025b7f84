// nk_precond.hip -- CG's fused updates (Krylov.jl cg!), the diagonal (Jacobi) right /
// left preconditioner with diag(J(u)) from the stencils' own tangent arithmetic, and ILU(0) of the
// stencil Jacobian (examples/bratu.jl:119-137's `ilu(collect(J))` on J's sparsity pattern): one
// work-group level sweep and the pipelined wavefront sweeps.  All bit-identical to the oracle.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "nk_stencil.hpp"

namespace nk {
namespace {

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

int launch_cg_update(nk_ctx* c, int64_t n, double alpha, double* x, double* r, const double* p, const double* Ap, Red* rr) {
    const int g = red_blocks(n);
    int fin;
    double* part = red_out(c, g, rr, &fin);
    return launch(c, "cg_update", 48.0 * n, [&] {
        hipLaunchKernelGGL(k_cg_update, dim3(g), dim3(kBlock), 0, c->stream, n, alpha, x, r, p, Ap, part, fin);
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
    const int g = wide_blocks(n);
    return launch(c, "cg_direction", 24.0 * (double)n,
                  [&] { hipLaunchKernelGGL(k_cg_direction, dim3(g), dim3(kBlock), 0, c->stream, n, beta, p, r); });
}

}  // namespace nk
