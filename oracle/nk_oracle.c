/*
 * nk_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity oracle and the CPU baseline).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU comparison.  The product path
 * (newtonkrylov.jl_amd/, libnkhip.so) never links, loads or falls back to it.
 *
 * What it is: a plain-C (OpenMP) restatement of the reference's hot path
 *   - Ariadne's inexact Newton driver       src/Ariadne.jl:288-372
 *   - Eisenstat-Walker / Fixed forcing       src/Ariadne.jl:185-217
 *   - the exact Jacobian-vector product      src/Ariadne.jl:48-57 (Enzyme Forward; here the
 *     hand-derived tangent of each residual), plus the FD operator of BASELINE.json's north star
 *   - Krylov.jl 0.10 gmres!/cg! (third-party, NOT present in /root/reference; pinned only by
 *     compat "0.10.1" in Project.toml:8,14 -- restated from its published algorithm, see
 *     SURVEY.md Appendix A.  Iterates and iteration counts are therefore "parity unpinned"
 *     against the reference; tests pin this oracle with the reference's own known answers
 *     (test/runtests.jl) and with independent numpy/scipy goldens in tests/golden/.)
 *   - residuals: 1D Bratu examples/bratu.jl:14-24, 2D heat diffusion! with bc_zero! /
 *     bc_periodic! (examples/heat_2D.jl:15-62) composed with G_Euler! / G_Midpoint! /
 *     G_Trapezoid! (examples/implicit.jl:8-37), and their build-defined generalisations
 *     2D Bratu and 3D heat.
 *
 * Layout: dense interior arrays, x fastest: idx = (k*ny + j)*nx + i (the same memory order as
 * the reference's column-major u[i,j]).  Zero-Dirichlet boundaries are applied by predication
 * (the reference writes zeros into ghost cells with bc_zero!, heat_2D.jl:28-38).
 *
 * Floating point: compiled with -ffp-contract=off so every stencil expression rounds exactly as
 * written (the reference's evaluation order, Julia does not contract).  BLAS-1 axpy uses fma()
 * explicitly (OpenBLAS daxpy, which Krylov.jl calls for dense vectors, is FMA based); the device
 * kernels use the same convention, so elementwise ops agree bit for bit.  Reductions are
 * deterministic (fixed chunking, independent of the thread count); OC_DEVRED (oc_set_devred) sums
 * the one-rank 2D GMRES reductions in exactly the device kernels' order instead, so whole restarted
 * histories compare bit for bit (tests/test_hip_devred.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#include <omp.h>

/* The correctly rounded exp shared with the HIP stencils (newtonkrylov.jl_amd/csrc/nk_exp.h): the
 * Bratu residual's lam * exp(u) (examples/bratu.jl:21) evaluates to the same double on both sides,
 * so the Bratu residual / JVP / FD operator are compared bit for bit like the heat kinds.  The exp
 * itself is pinned independently (tests/test_exp.py: mpmath at 200 bits on >= 10^6 inputs). */
#define NKX_FN static inline
#define NKX_SLOW_FN static
#define NKX_CONST static const
#include "nk_exp.h"
#ifdef NK_ORACLE_LIBM_EXP
/* The libm variant (oracle/_build/libnkoracle_libm.so, tests/test_oracle.py only): the same oracle with the
 * platform's exp (glibc: faithful, like Julia's Base.exp, not proven correctly rounded) -- so a regression in
 * the shared exp cannot hide behind device and oracle results that match because they share it. */
#define nk_exp(x) exp(x)
#endif

enum { OC_BRATU1D = 1, OC_BRATU2D = 2, OC_HEAT2D_EULER = 3, OC_HEAT3D_EULER = 4,
       OC_HEAT2D_MIDPOINT = 5, OC_HEAT3D_MIDPOINT = 6, OC_HEAT2D_TRAPEZOID = 7, OC_HEAT3D_TRAPEZOID = 8 };
enum { OC_BC_ZERO = 0, OC_BC_PERIODIC = 1 };
enum { OC_JV_EXACT = 0, OC_JV_FD = 1 };
enum { OC_FORCING_NONE = 0, OC_FORCING_FIXED = 1, OC_FORCING_EW = 2 };
enum { OC_ALGO_GMRES = 0, OC_ALGO_CG = 1, OC_ALGO_FGMRES = 2 };
/* right preconditioner N (Krylov.jl's `N`, ldiv = false):  DIAG z = d .* v (Jacobi: d = 1 ./ diag(J));
 * GMRES: z = gmres(J, v; itmax) -- the GmresPreconditioner of examples/bratu.jl:139-157 */
enum { OC_PRECOND_NONE = 0, OC_PRECOND_DIAG = 1, OC_PRECOND_GMRES = 3, OC_PRECOND_JACOBI = 4, OC_PRECOND_ILU0 = 5,
       OC_PRECOND_ILU = 6 /* Newton factory: ILU(0) of J(u) each step */ };

typedef struct {
    int32_t kind;           /* OC_PRECOND_DIAG / OC_PRECOND_GMRES */
    int32_t itmax;          /* GMRES: the inner solve's itmax */
    const double* diag;     /* DIAG: d;  ILU0: the pivots D~ */
    const struct oc_problem* P;  /* ILU0: J's off-diagonals */
} oc_precond;

typedef struct oc_problem {
    int32_t kind;
    int32_t bc;             /* OC_BC_ZERO (bc_zero!) or OC_BC_PERIODIC (bc_periodic!), heat kinds */
    int64_t nx, ny, nz;
    double hx, hy, hz;
    double lambda;          /* Bratu */
    double a, dt;           /* heat diffusivity and time step */
    const double* un;       /* heat: u_n (borrowed) */
    double alpha;           /* G_Midpoint! α (implicit.jl:17, default 0.5) */
} oc_problem;

typedef struct {
    int32_t memory;         /* Krylov workspace memory (default 20) */
    int32_t restart;        /* bool */
    int32_t reorthogonalization;
    int32_t itmax;          /* 0 => 2n */
    double atol, rtol;
    int32_t flexible;       /* fgmres! (Z_k = N V_k stored, x += Z y) instead of gmres! (x += N (V y)) */
    const oc_precond* N;    /* right preconditioner or NULL */
    const oc_precond* M;    /* left preconditioner (Krylov.jl's `M`, ldiv = false) or NULL */
} oc_krylov_opts;

typedef struct {
    int64_t niter;
    int32_t solved, inconsistent, breakdown, status;
    int64_t n_matvec;       /* mul!(J) calls incl. restart residuals */
} oc_krylov_stats;

typedef struct {
    double tol_rel, tol_abs;
    int32_t max_niter;
    int32_t forcing;        /* OC_FORCING_* */
    double eta_fixed, eta_max, gamma;
    int32_t algo;           /* OC_ALGO_* */
    int32_t jv_mode;        /* OC_JV_* */
    oc_krylov_opts krylov;
    int32_t rtol_user;      /* krylov_kwargs carries rtol: it wins over the forcing (Ariadne.jl:330-333) */
    int32_t precond;        /* N factory called per Newton step: OC_PRECOND_NONE / _JACOBI / _GMRES */
    int32_t precond_itmax;  /* OC_PRECOND_GMRES: GmresPreconditioner(J, itmax) */
    int32_t mprecond;       /* M factory called per Newton step (Ariadne.jl:327-329): same kinds as `precond` */
    int32_t mprecond_itmax;
} oc_newton_opts;

typedef struct {
    int64_t outer_iterations, inner_iterations;
    double n_res;
    int32_t solved;
    int64_t n_matvec, n_residual;
    double tol;
} oc_newton_stats;

static inline int64_t oc_n(const oc_problem* P) { return P->nx * P->ny * P->nz; }

/* ------------------------------------------------------------------ BLAS-1 (Krylov k* primitives) */
/* reduction chunk (fixed-order partial sums; oc_set_chunk changes the order to measure how much a
 * different summation order alone moves a result -- the GPU's reduction tree differs from this one) */
static int64_t OC_CHUNK = 8192;
void oc_set_chunk(int64_t c) { OC_CHUNK = c > 0 ? c : 8192; }

double oc_dot(int64_t n, const double* x, const double* y) {
    int64_t nch = (n + OC_CHUNK - 1) / OC_CHUNK;
    double* part = (double*)malloc(sizeof(double) * (size_t)(nch > 0 ? nch : 1));
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < nch; ++c) {
        int64_t lo = c * OC_CHUNK, hi = lo + OC_CHUNK < n ? lo + OC_CHUNK : n;
        double s = 0.0;
        for (int64_t i = lo; i < hi; ++i) s = fma(x[i], y[i], s);
        part[c] = s;
    }
    double s = 0.0;
    for (int64_t c = 0; c < nch; ++c) s += part[c];
    free(part);
    return s;
}
double oc_norm(int64_t n, const double* x) { return sqrt(oc_dot(n, x, x)); }

void oc_axpy(int64_t n, double s, const double* x, double* y) {   /* y += s x      (kaxpy!)  */
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) y[i] = fma(s, x[i], y[i]);
}
void oc_axpby(int64_t n, double s, const double* x, double t, double* y) { /* y = s x + t y (kaxpby!) */
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) y[i] = fma(t, y[i], s * x[i]);
}
void oc_scal(int64_t n, double s, double* x) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) x[i] = s * x[i];
}
void oc_copy(int64_t n, double* y, const double* x) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) y[i] = x[i];
}
void oc_fill(int64_t n, double* x, double v) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) x[i] = v;
}
void oc_divcopy(int64_t n, double* y, const double* x, double s) { /* y = x / s (kdivcopy!) */
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) y[i] = x[i] / s;
}
void oc_ref(int64_t n, double* x, double* y, double c, double s) { /* Givens on vectors (kref!) */
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        double xi = x[i], yi = y[i];
        x[i] = c * xi + s * yi;
        y[i] = s * xi - c * yi;
    }
}

/* ------------------------------------------------------------------ residuals */
/* ((p - 2c) + m) / (h*h): Julia's (u[i+1] - 2u[i] + u[i-1]) / Δx^2 (bratu.jl:19, heat_2D.jl:57-59) */
static inline double lap1(double c, double p, double m, double h) { return ((p - 2.0 * c) + m) / (h * h); }

#define AT(arr, i, j, k) ((arr)[((int64_t)(k) * ny + (j)) * nx + (i)])

static inline int oc_heat_dim(int kind) {
    return (kind == OC_HEAT2D_EULER || kind == OC_HEAT2D_MIDPOINT || kind == OC_HEAT2D_TRAPEZOID) ? 2 : 3;
}
static inline int oc_scheme(int kind) {  /* 0 G_Euler!, 1 G_Midpoint!, 2 G_Trapezoid! (implicit.jl:8-37) */
    if (kind == OC_HEAT2D_MIDPOINT || kind == OC_HEAT3D_MIDPOINT) return 1;
    if (kind == OC_HEAT2D_TRAPEZOID || kind == OC_HEAT3D_TRAPEZOID) return 2;
    return 0;
}

/* The 7 stencil positions (centre, +x, -x, +y, -y, +z, -z) of point (i,j,k): linear index, or -1 for
 * a zero ghost cell.  bc_zero! (heat_2D.jl:28-38) makes every ghost 0; bc_periodic! (heat_2D.jl:15-26)
 * copies the opposite interior edge into it, i.e. the neighbour index wraps around. */
static inline void stencil_idx(const oc_problem* P, int64_t i, int64_t j, int64_t k, int64_t q[7]) {
    const int64_t nx = P->nx, ny = P->ny, nz = P->nz;
    const int per = P->bc == OC_BC_PERIODIC;
    const int64_t ii[7] = {i, i + 1, i - 1, i, i, i, i};
    const int64_t jj[7] = {j, j, j, j + 1, j - 1, j, j};
    const int64_t kk[7] = {k, k, k, k, k, k + 1, k - 1};
    for (int s = 0; s < 7; ++s) {
        int64_t a = ii[s], b = jj[s], c = kk[s];
        if (per) {
            a = a < 0 ? a + nx : (a >= nx ? a - nx : a);
            b = b < 0 ? b + ny : (b >= ny ? b - ny : b);
            c = c < 0 ? c + nz : (c >= nz ? c - nz : c);
        }
        q[s] = (a < 0 || a >= nx || b < 0 || b >= ny || c < 0 || c >= nz) ? -1 : (c * ny + b) * nx + a;
    }
}

/* diffusion!'s Laplacian sum at the centre of f[7] (heat_2D.jl:55-60; 3D: ((x + y) + z)) */
static inline double heat_lap(const oc_problem* P, const double f[7], int dim) {
    double l = lap1(f[0], f[1], f[2], P->hx) + lap1(f[0], f[3], f[4], P->hy);
    if (dim == 3) l = l + lap1(f[0], f[5], f[6], P->hz);
    return l;
}

/* G(u + eps v) at one point of a heat problem (v == NULL: G(u)).  du = a * lap(.):
 *   G_Euler!     (implicit.jl:8-13)  res = (u_n + Δt du(w)) - w
 *   G_Midpoint!  (implicit.jl:17-25) m = α u_n + (1 - α) w (elementwise, bc! applied to m);
 *                                    res = (u_n + Δt du(m)) - w
 *   G_Trapezoid! (implicit.jl:29-37) res = (u_n + (Δt/2)(du(u_n) + du(w))) - w               */
static inline double heat_point(const oc_problem* P, const double* u, const double* v, double eps, int64_t i,
                                int64_t j, int64_t k) {
    int64_t q[7];
    stencil_idx(P, i, j, k, q);
    const int dim = oc_heat_dim(P->kind), sch = oc_scheme(P->kind);
    const int ns = dim == 3 ? 7 : 5;
    double w[7] = {0}, un[7] = {0}, m[7] = {0};
    for (int s = 0; s < ns; ++s) {
        if (q[s] < 0) continue;
        w[s] = v ? u[q[s]] + eps * v[q[s]] : u[q[s]];
        un[s] = P->un[q[s]];
        m[s] = P->alpha * un[s] + (1.0 - P->alpha) * w[s];
    }
    if (sch == 1) return (un[0] + P->dt * (P->a * heat_lap(P, m, dim))) - w[0];
    if (sch == 2) return (un[0] + (P->dt / 2.0) * (P->a * heat_lap(P, un, dim) + P->a * heat_lap(P, w, dim))) - w[0];
    return (un[0] + P->dt * (P->a * heat_lap(P, w, dim))) - w[0];
}

/* value of w at (i,j,k) with zero Dirichlet outside, where w = u (+ eps*v when v != NULL) */
static inline double wval(const double* u, const double* v, double eps, int64_t nx, int64_t ny, int64_t nz,
                          int64_t i, int64_t j, int64_t k) {
    if (i < 0 || i >= nx || j < 0 || j >= ny || k < 0 || k >= nz) return 0.0;
    double x = AT(u, i, j, k);
    if (v) x = x + eps * AT(v, i, j, k);
    return x;
}

/* F(w) at one point, w = u + eps*v (v==NULL: w = u) */
static inline double point_residual(const oc_problem* P, const double* u, const double* v, double eps,
                                    int64_t i, int64_t j, int64_t k) {
    const int64_t nx = P->nx, ny = P->ny, nz = P->nz;
    double c = wval(u, v, eps, nx, ny, nz, i, j, k);
    switch (P->kind) {
    case OC_BRATU1D: {
        double l = wval(u, v, eps, nx, ny, nz, i - 1, j, k), r = wval(u, v, eps, nx, ny, nz, i + 1, j, k);
        return lap1(c, r, l, P->hx) + P->lambda * nk_exp(c);
    }
    case OC_BRATU2D: {
        double e = wval(u, v, eps, nx, ny, nz, i + 1, j, k), w = wval(u, v, eps, nx, ny, nz, i - 1, j, k);
        double n = wval(u, v, eps, nx, ny, nz, i, j + 1, k), s = wval(u, v, eps, nx, ny, nz, i, j - 1, k);
        return (lap1(c, e, w, P->hx) + lap1(c, n, s, P->hy)) + P->lambda * nk_exp(c);
    }
    default:
        return heat_point(P, u, v, eps, i, j, k);
    }
}

void oc_residual(const oc_problem* P, double* res, const double* u) {
    const int64_t nx = P->nx, ny = P->ny, nz = P->nz;
#pragma omp parallel for collapse(2) schedule(static)
    for (int64_t k = 0; k < nz; ++k)
        for (int64_t j = 0; j < ny; ++j)
            for (int64_t i = 0; i < nx; ++i) AT(res, i, j, k) = point_residual(P, u, NULL, 0.0, i, j, k);
}

/* exact JVP of a heat problem: the forward-mode tangent Enzyme computes through G! ∘ diffusion!.
 * u_n and du are constants (zero shadows), so 0 + x = x throughout:
 *   Euler     Δt (a lap(v)) - v
 *   Midpoint  Δt (a lap((1 - α) v)) - v      (the shadow of α u_n + (1 - α) u is (1 - α) v)
 *   Trapezoid (Δt/2) (a lap(v)) - v          (the shadow of du(u_n) is 0)                        */
static inline double heat_tangent(const oc_problem* P, const double* v, int64_t i, int64_t j, int64_t k) {
    int64_t q[7];
    stencil_idx(P, i, j, k, q);
    const int dim = oc_heat_dim(P->kind), sch = oc_scheme(P->kind);
    const int ns = dim == 3 ? 7 : 5;
    double f[7] = {0};
    for (int s = 0; s < ns; ++s) {
        if (q[s] < 0) continue;
        f[s] = sch == 1 ? (1.0 - P->alpha) * v[q[s]] : v[q[s]];
    }
    const double vc = v[q[0]];
    if (sch == 2) return (P->dt / 2.0) * (P->a * heat_lap(P, f, dim)) - vc;
    return P->dt * (P->a * heat_lap(P, f, dim)) - vc;
}

/* exact JVP: the forward-mode tangent Enzyme computes for each residual (Ariadne.jl:48-57) */
void oc_jv_exact(const oc_problem* P, double* out, const double* u, const double* v) {
    const int64_t nx = P->nx, ny = P->ny, nz = P->nz;
#pragma omp parallel for collapse(2) schedule(static)
    for (int64_t k = 0; k < nz; ++k)
        for (int64_t j = 0; j < ny; ++j)
            for (int64_t i = 0; i < nx; ++i) {
                double c = AT(v, i, j, k), r;
                double e = wval(v, NULL, 0, nx, ny, nz, i + 1, j, k), w = wval(v, NULL, 0, nx, ny, nz, i - 1, j, k);
                switch (P->kind) {
                case OC_BRATU1D:
                    r = lap1(c, e, w, P->hx) + P->lambda * (nk_exp(AT(u, i, j, k)) * c);
                    break;
                case OC_BRATU2D: {
                    double n = wval(v, NULL, 0, nx, ny, nz, i, j + 1, k), s = wval(v, NULL, 0, nx, ny, nz, i, j - 1, k);
                    r = (lap1(c, e, w, P->hx) + lap1(c, n, s, P->hy)) + P->lambda * (nk_exp(AT(u, i, j, k)) * c);
                    break;
                }
                default:
                    r = heat_tangent(P, v, i, j, k);
                }
                AT(out, i, j, k) = r;
            }
}

/* FD JVP (BASELINE.json north star): out = (F(u + eps v) - F0) / eps */
void oc_jv_fd(const oc_problem* P, double* out, const double* u, const double* v, const double* F0, double eps) {
    const int64_t nx = P->nx, ny = P->ny, nz = P->nz;
#pragma omp parallel for collapse(2) schedule(static)
    for (int64_t k = 0; k < nz; ++k)
        for (int64_t j = 0; j < ny; ++j)
            for (int64_t i = 0; i < nx; ++i)
                AT(out, i, j, k) = (point_residual(P, u, v, eps, i, j, k) - AT(F0, i, j, k)) / eps;
}

/* eps = sqrt(eps_mach) * max(1, ||u||) / ||v||  (SURVEY.md §6 probe; ||v|| := 1 for Arnoldi basis vectors) */
double oc_fd_eps(double unorm, double vnorm) { return sqrt(DBL_EPSILON) * fmax(1.0, unorm) / vnorm; }

typedef struct {
    const oc_problem* P;
    int mode;
    const double* u;
    const double* F0;
    double unorm;
    int64_t n_matvec;
} oc_op;

static void op_apply(oc_op* A, double* out, const double* v, double vnorm) {
    A->n_matvec++;
    if (A->mode == OC_JV_EXACT) {
        oc_jv_exact(A->P, out, A->u, v);
    } else {
        if (vnorm < 0) vnorm = oc_norm(oc_n(A->P), v);
        if (vnorm == 0.0) { oc_fill(oc_n(A->P), out, 0.0); return; }
        oc_jv_fd(A->P, out, A->u, v, A->F0, oc_fd_eps(A->unorm, vnorm));
    }
}

/* ------------------------------------------------------------------ the device's summation order (OC_DEVRED)
 * Test infrastructure for VERDICT r05 item 5: the GMRES reductions summed in EXACTLY the order the
 * product's kernels sum them (one rank, 2D kinds), so restarted FD-GMRES histories compare bit for bit at
 * any length instead of drifting apart by reduction order.  Every tree below restates one device
 * reduction (newtonkrylov.jl_amd/csrc/, file named at each); the per-element products are the same fma()
 * the default mode uses.  Hardware parameters: the CU count (the resident sweep's grid, 256 on MI355X)
 * and the sweep's LDS slots per thread (39) -- the test asserts the device reports the same grid.
 *   wave:  wave_sum, a 64-lane butterfly (v += shfl_xor(v, o), o = 32 .. 1; lane 0)   nk_device.hpp
 *   block: block_sum<256>, four wave sums added in wave order                        nk_device.hpp
 *   RI:    reduce_input / k_finalize: thread t sums in[t], in[t + 256], ... then block nk_device.hpp
 *   chunk: k_dot / k_sumsq / k_mgs_pass / k_update_x: block b owns a 256-multiple chunk of the
 *          double2 elements, thread t its elements t, t + 256, ... (x then y component) nk_kernels.hip
 *   tiles: k_st2d: tile (tx, ty) = 256 VEC columns x `rows` rows, thread t its VEC columns row by
 *          row; partial index = tile index                                             nk_stencil.hpp
 *   sweep: k_mgs_res: block b owns slots [b S / G, (b + 1) S / G) of 256 double2; partials summed by
 *          one polling wave (lane l: blocks l, 64 + l, 128 + l, 192 + l, then a wave sum) nk_resident.hip */
static int OC_DEVRED = 0, OC_DEV_CUS = 256, OC_DEV_RL = 39;
/* the ranks' decomposition (px x py x pz blocks, rank = (iz py + iy) px + ix, every axis split as
 * ariadne_hip.block / slab split it; 2D slabs: 1 x R x 1) and whether their sweeps run resident (ranks
 * sharing one GPU do not) -- each rank's partials in its own block's order, the ranks' sums added in rank
 * order as the peer mailbox adds them (mb_recv) */
static int OC_DEV_PX = 1, OC_DEV_PY = 1, OC_DEV_PZ = 1, OC_DEV_RESIDENT = 1;
static double OC_DEV_BNORM = 0.0;  /* > 0: the Newton driver's ||F(u)||, which the device solve takes as ||b|| */
/* the device evaluates the residual as a USER problem (NK_USER*, nk_user.cpp): the callback's F, then
 * k_user_epi's scalar chunks for every reduction a built-in stencil sums over its tiles */
static int OC_DEV_USER = 0;
void oc_set_devred(int on, int cus, int rl) {
    OC_DEVRED = on;
    OC_DEV_CUS = cus > 0 && cus <= 256 ? cus : 256;
    OC_DEV_RL = rl >= 0 ? rl : 39;
    OC_DEV_PX = OC_DEV_PY = OC_DEV_PZ = OC_DEV_RESIDENT = 1;
    OC_DEV_USER = 0;
}
void oc_set_devred_user(int user) { OC_DEV_USER = user != 0; }
void oc_set_devred_ranks(int px, int py, int pz, int resident) {
    OC_DEV_PX = px > 0 ? px : 1;
    OC_DEV_PY = py > 0 ? py : 1;
    OC_DEV_PZ = pz > 0 ? pz : 1;
    OC_DEV_RESIDENT = resident != 0;
}
int oc_get_devred(void) { return OC_DEVRED; }

static double dr_wave(const double* v) {
    double a[64], b[64];
    memcpy(a, v, sizeof a);
    for (int o = 32; o > 0; o >>= 1) {
        for (int l = 0; l < 64; ++l) b[l] = a[l] + a[l ^ o];
        memcpy(a, b, sizeof a);
    }
    return a[0];
}
static double dr_block(const double* acc) {
    double r = dr_wave(acc);
    for (int w = 1; w < 4; ++w) r += dr_wave(acc + 64 * w);
    return r;
}
double oc_dr_ri(const double* in, int64_t len) {
    double acc[256];
    for (int t = 0; t < 256; ++t) {
        double s = 0.0;
        for (int64_t m = t; m < len; m += 256) s += in[m];
        acc[t] = s;
    }
    return dr_block(acc);
}
static int64_t dr_red_blocks(int64_t n) {  /* red_blocks: >= 4 double2 per thread, at most 2048 */
    int64_t g = (n + 2LL * 256 * 4 - 1) / (2LL * 256 * 4);
    return g < 1 ? 1 : (g > 2048 ? 2048 : g);
}
static int64_t dr_wide_blocks(int64_t n) {  /* wide_blocks: >= 2 double2 per thread, at most kRedCap - 2 */
    int64_t g = (n + 2LL * 256 * 2 - 1) / (2LL * 256 * 2);
    return g < 1 ? 1 : (g > 16382 ? 16382 : g);
}
/* the chunked streaming kernels' partials of sum x_i y_i over G blocks (y == NULL: x_i^2) */
void oc_dr_chunk_parts(int64_t n, const double* x, const double* y, int64_t G, double* parts) {
    if (!y) y = x;
    const int64_t n2 = n >> 1, per = ((n2 + G - 1) / G + 255) / 256 * 256;
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < G; ++b) {
        double acc[256] = {0.0};
        const int64_t lo = b * per, hi = lo + per < n2 ? lo + per : n2;
        for (int64_t i = lo; i < hi; ++i) {
            const int t = (int)((i - lo) & 255);
            acc[t] = fma(x[2 * i], y[2 * i], acc[t]);
            acc[t] = fma(x[2 * i + 1], y[2 * i + 1], acc[t]);
        }
        if ((n & 1) && b == 0) acc[0] = fma(x[n - 1], y[n - 1], acc[0]);
        parts[b] = dr_block(acc);
    }
}
/* k_cg_update's partials: the same chunks over the n SCALAR elements (NK_CHUNKED(i, n), nk_precond.hip) */
static double dr_chunk1(int64_t n, const double* x, const double* y, int64_t G) {
    if (!y) y = x;
    const int64_t per = ((n + G - 1) / G + 255) / 256 * 256;
    double* parts = (double*)malloc(sizeof(double) * (size_t)G);
    for (int64_t b = 0; b < G; ++b) {
        double acc[256] = {0.0};
        const int64_t lo = b * per, hi = lo + per < n ? lo + per : n;
        for (int64_t i = lo; i < hi; ++i) acc[(i - lo) & 255] = fma(x[i], y[i], acc[(i - lo) & 255]);
        parts[b] = dr_block(acc);
    }
    const double r = oc_dr_ri(parts, G);
    free(parts);
    return r;
}
static double dr_chunk(int64_t n, const double* x, const double* y, int64_t G) {
    double* parts = (double*)malloc(sizeof(double) * (size_t)G);
    oc_dr_chunk_parts(n, x, y, G, parts);
    const double r = oc_dr_ri(parts, G);
    free(parts);
    return r;
}
/* k_st2d's tile geometry (launch_stencil_ex, nk_kernels.hip: about 1024 tiles of 8 .. 32 rows) */
static void dr_tiles2d(int64_t nx, int64_t ny, int* vec, int64_t* tiles_x, int64_t* rows, int64_t* tiles_y) {
    *vec = nx % 2 == 0 ? 2 : 1;
    *tiles_x = (nx + 256 * *vec - 1) / (256 * *vec);
    int64_t r = (ny * *tiles_x + 1023) / 1024;
    if (r > 32) r = 32;
    if (r < 8) r = 8;
    const int64_t cap_rows = (ny * *tiles_x + (16384 - 3)) / (16384 - 2);
    if (r < cap_rows) r = cap_rows;
    if (r > ny) r = ny;
    *rows = r;
    *tiles_y = (ny + r - 1) / r;
}
int64_t oc_dr_tile_parts2d(int64_t nx, int64_t ny, const double* x, const double* y, double* parts) {
    if (!y) y = x;
    int vec;
    int64_t tx_n, rows, ty_n;
    dr_tiles2d(nx, ny, &vec, &tx_n, &rows, &ty_n);
    if (!parts) return tx_n * ty_n;
#pragma omp parallel for schedule(static)
    for (int64_t tl = 0; tl < tx_n * ty_n; ++tl) {
        const int64_t tx = tl % tx_n, ty = tl / tx_n;
        const int64_t y0 = ty * rows, y1 = y0 + rows < ny ? y0 + rows : ny;
        double acc[256] = {0.0};
        for (int t = 0; t < 256; ++t) {
            const int64_t x0 = tx * 256 * vec + (int64_t)t * vec;
            if (x0 >= nx) continue;
            double a = 0.0;
            for (int64_t j = y0; j < y1; ++j)
                for (int k = 0; k < vec; ++k) a = fma(x[j * nx + x0 + k], y[j * nx + x0 + k], a);
            acc[t] = a;
        }
        parts[tl] = dr_block(acc);
    }
    return tx_n * ty_n;
}
/* k_st3l's tiles (launch_stencil_ex, nk_kernels.hip): 4 rows (one per wave) x 64 VEC columns, z-chunks of
 * `planes` (blocks: 16; else about 8192 tiles, at least 16), partial index tz tiles_x tiles_y + ty tiles_x + tx;
 * thread (wave w, lane l) sums its VEC points of row ty 4 + w plane by plane upward */
int64_t oc_dr_tile_parts3d(int64_t nx, int64_t ny, int64_t nz, int blk, const double* x, const double* y, double* parts) {
    if (!y) y = x;
    const int vec = nx % 2 == 0 ? 2 : 1;
    const int64_t tx_n = (nx + 64 * vec - 1) / (64 * vec), ty_n = (ny + 3) / 4, tpl = tx_n * ty_n;
    int64_t planes = (nz * tpl + 8191) / 8192;
    if (planes < 16 || blk) planes = 16;
    if (planes > nz) planes = nz;
    const int64_t nzc = (nz + planes - 1) / planes, pl = nx * ny;
    if (!parts) return tpl * nzc;
#pragma omp parallel for schedule(static)
    for (int64_t tl = 0; tl < tpl * nzc; ++tl) {
        const int64_t tz = tl / tpl, ty = (tl % tpl) / tx_n, tx = tl % tx_n;
        const int64_t z0 = tz * planes, z1 = z0 + planes < nz ? z0 + planes : nz;
        double acc[256] = {0.0};
        for (int t = 0; t < 256; ++t) {
            const int64_t j = ty * 4 + t / 64, x0 = tx * 64 * vec + (int64_t)(t % 64) * vec;
            if (x0 >= nx || j >= ny) continue;
            double a = 0.0;
            for (int64_t k = z0; k < z1; ++k)
                for (int q = 0; q < vec; ++q) a = fma(x[k * pl + j * nx + x0 + q], y[k * pl + j * nx + x0 + q], a);
            acc[t] = a;
        }
        parts[tl] = dr_block(acc);
    }
    return tpl * nzc;
}
/* k_st1d: one point per thread, one partial per 256-point block */
int64_t oc_dr_tile_parts1d(int64_t nx, const double* x, const double* y, double* parts) {
    if (!y) y = x;
    const int64_t G = (nx + 255) / 256;
    if (!parts) return G;
    for (int64_t b = 0; b < G; ++b) {
        double acc[256] = {0.0};
        for (int t = 0; t < 256 && b * 256 + t < nx; ++t) acc[t] = fma(x[b * 256 + t], y[b * 256 + t], 0.0);
        parts[b] = dr_block(acc);
    }
    return G;
}
/* one rank's sum of its stencil launch's tile partials (reduce_input over the tiles) */
static double dr_tiles_local(int dim, int64_t nx, int64_t ny, int64_t nz, int blk, const double* x, const double* y) {
    const int64_t nt = dim == 3 ? oc_dr_tile_parts3d(nx, ny, nz, blk, x, y, NULL)
                       : dim == 2 ? oc_dr_tile_parts2d(nx, ny, x, y, NULL) : oc_dr_tile_parts1d(nx, x, y, NULL);
    double* parts = (double*)malloc(sizeof(double) * (size_t)nt);
    if (dim == 3) oc_dr_tile_parts3d(nx, ny, nz, blk, x, y, parts);
    else if (dim == 2) oc_dr_tile_parts2d(nx, ny, x, y, parts);
    else oc_dr_tile_parts1d(nx, x, y, parts);
    const double r = oc_dr_ri(parts, nt);
    free(parts);
    return r;
}
/* the resident sweep (launch_mgs_sweep, nk_resident.hip): does it run for np passes over n points? */
static int dr_sweep_applies(int64_t n, int np) {
    if (np < 2 || np > 64 || (n & 1)) return 0;
    const int64_t G = OC_DEV_CUS, n2 = n >> 1, ns = (n2 + 255) / 256;
    const int64_t whole = ns / G - (n2 % 256 != 0 ? 1 : 0);
    if (whole < 1) return 0;
    const int64_t slots = whole < (1 << 20) ? whole : (1 << 20);
    int64_t rl = slots < OC_DEV_RL ? slots : OC_DEV_RL, rv = slots - rl, pick = 0;
    static const int kRv[] = {89, 64, 48, 32, 25, 16, 0};
    for (int i = 0; i < 7; ++i)
        if (kRv[i] <= rv && kRv[i] <= slots) { pick = kRv[i]; break; }
    rv = pick;
    if (rl > slots - rv) rl = slots - rv;
    const int64_t chunk = ns / G > 1 ? ns / G : 1;
    return (double)(rv + rl) / (double)chunk >= 0.1;
}
void oc_dr_sweep_parts(int64_t n, const double* x, const double* y, int64_t G, double* parts) {
    if (!y) y = x;
    const int64_t n2 = n >> 1, ns = (n2 + 255) / 256;
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < G; ++b) {
        double acc[256] = {0.0};
        const int64_t lo = b * ns / G * 256, hi0 = (b + 1) * ns / G * 256, hi = hi0 < n2 ? hi0 : n2;
        for (int64_t i = lo; i < hi; ++i) {
            const int t = (int)((i - lo) & 255);
            acc[t] = fma(x[2 * i], y[2 * i], acc[t]);
            acc[t] = fma(x[2 * i + 1], y[2 * i + 1], acc[t]);
        }
        parts[b] = dr_block(acc);
    }
}
double oc_dr_poll1(const double* parts, int64_t G) {
    double v[64];
    for (int l = 0; l < 64; ++l) {
        double p = 0.0;
        for (int j = 0; j < 4; ++j) p += (64 * j + l < G) ? parts[64 * j + l] : 0.0;
        v[l] = p;
    }
    return dr_wave(v);
}
static double dr_sweep(int64_t n, const double* x, const double* y) {
    const int64_t G = OC_DEV_CUS;
    double parts[256];
    oc_dr_sweep_parts(n, x, y, G, parts);
    return oc_dr_poll1(parts, G);
}
/* devred applies to GMRES / FGMRES / CG, preconditioned or not (Jacobi, ILU(0), the GMRES preconditioner) */
static int dr_on(const oc_problem* P) {
    (void)P;
    return OC_DEVRED;
}
enum { DR_RED = 0, DR_WIDE = 1, DR_TILES = 2, DR_PASS = 3, DR_RED1 = 4 };
static double dr_reduce(const oc_problem* P, int kind, const double* x, const double* y, int np);
/* ||z||^2 of z = N v as apply_precond (nk_krylov.cpp) sums it: fused into k_diag_apply's scalar chunks for a
 * diagonal N, k_sumsq after the ILU(0) solve / the inner GMRES */
static double dr_prec_norm2(const oc_problem* P, const oc_precond* N, const double* z) {
    return dr_reduce(P, N->kind == OC_PRECOND_DIAG ? DR_RED1 : DR_RED, z, NULL, 0);
}
/* one reduction of sum x_i y_i (y NULL: x_i^2) over the global grid, as the ranks compute it: each rank its
 * block's tree (DR_RED: k_sumsq / k_dot over red_blocks; DR_WIDE: k_update_x's wide_blocks; DR_TILES: the
 * stencil's tiles; DR_PASS: an MGS pass of an np-pass step -- the resident sweep where it runs, else
 * k_mgs_pass's chunks), then the ranks' values added in rank order from 0.0 (mb_recv) */
static double dr_reduce(const oc_problem* P, int kind, const double* x, const double* y, int np) {
    const int dim = P->kind == OC_BRATU1D ? 1 : (P->kind == OC_BRATU2D || oc_heat_dim(P->kind) == 2 ? 2 : 3);
    const int px = OC_DEV_PX, py = dim >= 2 ? OC_DEV_PY : 1, pz = dim == 3 ? OC_DEV_PZ : 1;
    const int64_t NX = P->nx, NY = dim >= 2 ? P->ny : 1, NZ = dim == 3 ? P->nz : 1;
    const int R = px * py * pz, blk = dim == 3 && px * py > 1;
    double total = 0.0;
    double *lx = NULL, *ly = NULL;
    for (int r = 0; r < R; ++r) {
        const int ix = r % px, iy = (r / px) % py, iz = r / (px * py);
        int64_t o[3], m[3];
        const int64_t N[3] = {NX, NY, NZ};
        const int idx[3] = {ix, iy, iz}, parts_[3] = {px, py, pz};
        for (int a = 0; a < 3; ++a) {  /* split as ariadne_hip.block / slab: the first N % p parts one larger */
            const int64_t base = N[a] / parts_[a], extra = N[a] % parts_[a];
            m[a] = base + (idx[a] < extra ? 1 : 0);
            o[a] = idx[a] * base + (idx[a] < extra ? idx[a] : extra);
        }
        const int64_t nl = m[0] * m[1] * m[2];
        const double *xs = x, *ys = y;
        if (R > 1) {  /* this rank's block, x fastest */
            lx = (double*)realloc(lx, sizeof(double) * (size_t)nl);
            if (y) ly = (double*)realloc(ly, sizeof(double) * (size_t)nl);
            for (int64_t k = 0; k < m[2]; ++k)
                for (int64_t j = 0; j < m[1]; ++j) {
                    const int64_t g = ((o[2] + k) * NY + o[1] + j) * NX + o[0], l = (k * m[1] + j) * m[0];
                    memcpy(lx + l, x + g, sizeof(double) * (size_t)m[0]);
                    if (y) memcpy(ly + l, y + g, sizeof(double) * (size_t)m[0]);
                }
            xs = lx;
            ys = y ? ly : NULL;
        }
        double v;
        if (kind == DR_TILES && OC_DEV_USER) v = dr_chunk1(nl, xs, ys, dr_red_blocks(nl));  /* k_user_epi */
        else if (kind == DR_TILES) v = dr_tiles_local(dim, m[0], m[1], m[2], blk, xs, ys);
        else if (kind == DR_WIDE) v = dr_chunk(nl, xs, ys, dr_wide_blocks(nl));
        else if (kind == DR_RED1) v = dr_chunk1(nl, xs, ys, dr_red_blocks(nl));
        else if (kind == DR_PASS && OC_DEV_RESIDENT && dr_sweep_applies(nl, np)) v = dr_sweep(nl, xs, ys ? ys : xs);
        else v = dr_chunk(nl, xs, ys, dr_red_blocks(nl));
        total = R > 1 ? total + v : v;
    }
    free(lx);
    free(ly);
    return total;
}

/* ------------------------------------------------------------------ Krylov.jl sym_givens (real) */
static inline double sgn(double x) { return (x > 0) - (x < 0); }
void oc_sym_givens(double a, double b, double* c, double* s, double* rho) {
    if (b == 0.0) {
        *c = (a == 0.0) ? 1.0 : sgn(a);
        *s = 0.0;
        *rho = fabs(a);
    } else if (a == 0.0) {
        *c = 0.0;
        *s = sgn(b);
        *rho = fabs(b);
    } else if (fabs(b) > fabs(a)) {
        double t = a / b;
        *s = sgn(b) / sqrt(1.0 + t * t);
        *c = *s * t;
        *rho = b / *s;
    } else {
        double t = b / a;
        *c = sgn(a) / sqrt(1.0 + t * t);
        *s = *c * t;
        *rho = a / *c;
    }
}

/* diag(J(u)): the exact tangent of each residual on the unit vector e_i (the diagonal of collect(J),
 * src/Ariadne.jl:140-162): centre field 1 -- (1 - α) for G_Midpoint! -- every neighbour 0 */
void oc_jacobian_diag(const oc_problem* P, double* out, const double* u, int reciprocal) {
    const int64_t n = oc_n(P);
    const int heat = P->kind >= OC_HEAT2D_EULER && P->kind <= OC_HEAT3D_TRAPEZOID;
    const int dim = P->kind == OC_BRATU1D ? 1 : (P->kind == OC_BRATU2D ? 2 : oc_heat_dim(P->kind));
    const int sch = heat ? oc_scheme(P->kind) : 0;
    const double c = sch == 1 ? (1.0 - P->alpha) * 1.0 : 1.0;
    double lsum = lap1(c, 0.0, 0.0, P->hx);
    if (dim >= 2) lsum = lsum + lap1(c, 0.0, 0.0, P->hy);
    if (dim == 3) lsum = lsum + lap1(c, 0.0, 0.0, P->hz);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        double d;
        if (!heat) d = lsum + P->lambda * (nk_exp(u[i]) * 1.0);
        else if (sch == 2) d = (P->dt / 2.0) * (P->a * lsum) - 1.0;
        else d = P->dt * (P->a * lsum) - 1.0;
        out[i] = reciprocal ? 1.0 / d : d;
    }
}

int oc_gmres(oc_op* A, const double* b, double* x, const oc_krylov_opts* o, oc_krylov_stats* st,
             double* hist, int64_t hist_cap, int64_t* hist_len);

/* ILU(0) of J in natural order (x fastest) on J's own pattern -- `ilu(collect(J))` of
 * examples/bratu.jl:119-137 without fill (for the 1D tridiagonal J this is the exact LU).  IKJ
 * elimination: for the 3/5/7-point stencil it only updates the diagonal,
 *   D~_i = ((a_ii - (c_z / D~_b) c_z) - (c_y / D~_s) c_y) - (c_x / D~_w) c_x,
 * lower neighbours in increasing index order; c_* = J's constant off-diagonal entry per axis (the
 * exact tangent at i of the unit vector on the neighbour: f / h^2, f = 1 or G_Midpoint!'s 1 - α). */
static double ilu_offdiag(const oc_problem* P, double h) {
    const int heat = P->kind >= OC_HEAT2D_EULER && P->kind <= OC_HEAT3D_TRAPEZOID;
    const int sch = heat ? oc_scheme(P->kind) : 0;
    const double f = sch == 1 ? (1.0 - P->alpha) * 1.0 : 1.0;
    const double lsum = ((f - 2.0 * 0.0) + 0.0) / (h * h);
    if (!heat) return lsum;
    return (sch == 2 ? P->dt / 2.0 : P->dt) * (P->a * lsum) - 0.0;
}
static int oc_dim(const oc_problem* P) {
    return P->kind == OC_BRATU1D ? 1 : (P->kind == OC_BRATU2D ? 2 : oc_heat_dim(P->kind));
}
void oc_ilu0_factor(const oc_problem* P, const double* u, double* d) {
    const int64_t nx = P->nx, ny = P->ny, nz = P->nz;
    const int dim = oc_dim(P);
    const double cx = ilu_offdiag(P, P->hx), cy = dim >= 2 ? ilu_offdiag(P, P->hy) : 0.0,
                 cz = dim == 3 ? ilu_offdiag(P, P->hz) : 0.0;
    oc_jacobian_diag(P, d, u, 0);
    for (int64_t k = 0; k < nz; ++k)
        for (int64_t j = 0; j < ny; ++j)
            for (int64_t i = 0; i < nx; ++i) {
                const int64_t q = (k * ny + j) * nx + i;
                double a = d[q];
                if (k > 0) a = a - (cz / d[q - nx * ny]) * cz;
                if (j > 0) a = a - (cy / d[q - nx]) * cy;
                if (i > 0) a = a - (cx / d[q - 1]) * cx;
                d[q] = a;
            }
}
/* z = U^-1 L^-1 v */
void oc_ilu0_solve(const oc_problem* P, const double* d, double* z, const double* v) {
    const int64_t nx = P->nx, ny = P->ny, nz = P->nz, n = nx * ny * nz;
    const int dim = oc_dim(P);
    const double cx = ilu_offdiag(P, P->hx), cy = dim >= 2 ? ilu_offdiag(P, P->hy) : 0.0,
                 cz = dim == 3 ? ilu_offdiag(P, P->hz) : 0.0;
    for (int64_t q = 0; q < n; ++q) {
        const int64_t i = q % nx, j = (q / nx) % ny, k = q / (nx * ny);
        double a = v[q];
        if (k > 0) a = a - (cz / d[q - nx * ny]) * z[q - nx * ny];
        if (j > 0) a = a - (cy / d[q - nx]) * z[q - nx];
        if (i > 0) a = a - (cx / d[q - 1]) * z[q - 1];
        z[q] = a;
    }
    for (int64_t q = n - 1; q >= 0; --q) {
        const int64_t i = q % nx, j = (q / nx) % ny, k = q / (nx * ny);
        double a = z[q];
        if (i + 1 < nx) a = a - cx * z[q + 1];
        if (j + 1 < ny) a = a - cy * z[q + nx];
        if (k + 1 < nz) a = a - cz * z[q + nx * ny];
        z[q] = a / d[q];
    }
}

/* z = N v */
static void prec_apply(oc_op* A, const oc_precond* N, double* z, const double* v) {
    const int64_t n = oc_n(A->P);
    if (N->kind == OC_PRECOND_DIAG) {
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < n; ++i) z[i] = N->diag[i] * v[i];
    } else if (N->kind == OC_PRECOND_ILU0) {
        oc_ilu0_solve(N->P ? N->P : A->P, N->diag, z, v);
    } else { /* mul!(y, P::GmresPreconditioner, x): sol, _ = gmres(P.J, x; P.itmax); copyto!(y, sol) -- Krylov's
                gmres defaults: memory 20, no restart, atol = rtol = √eps, x0 = 0 */
        oc_krylov_opts io = {20, 0, 0, N->itmax, sqrt(DBL_EPSILON), sqrt(DBL_EPSILON), 0, NULL, NULL};
        oc_krylov_stats is;
        memset(&is, 0, sizeof is);
        oc_gmres(A, v, z, &io, &is, NULL, 0, NULL);
    }
}

/* ------------------------------------------------------------------ GMRES / FGMRES (Krylov.jl 0.10 gmres! / fgmres!)
 * Left preconditioner M (ldiv = false): r0 = M (b - A x), the Arnoldi vector q = M A (N V_k), and
 * beta / the stopping test measure the preconditioned residual; with M = I, r0 === w and q === w. */
static void* xrealloc(void* p, size_t sz) { void* q = realloc(p, sz); if (!q) abort(); return q; }

int oc_gmres(oc_op* A, const double* b, double* x, const oc_krylov_opts* o, oc_krylov_stats* st,
             double* hist, int64_t hist_cap, int64_t* hist_len) {
    const int64_t n = oc_n(A->P);
    int mem = o->memory > 0 ? o->memory : 20;
    const int restart = o->restart, reorth = o->reorthogonalization;
    int64_t itmax = o->itmax;
    int64_t nh = 0;
    const int64_t nmv0 = A->n_matvec;
#define PUSH_HIST(v) do { if (hist && nh < hist_cap) hist[nh] = (v); nh++; } while (0)

    double* w = (double*)malloc(sizeof(double) * n);
    double* xr = restart ? (double*)malloc(sizeof(double) * n) : x;
    const oc_precond* N = (o->N && o->N->kind != OC_PRECOND_NONE) ? o->N : NULL;
    const oc_precond* M = (o->M && o->M->kind != OC_PRECOND_NONE) ? o->M : NULL;
    double* r0 = M ? (double*)malloc(sizeof(double) * n) : w; /* r0 = M w */
    double* q = M ? (double*)malloc(sizeof(double) * n) : w;  /* q = M A p */
    const int flex = N && o->flexible;
    double* pv = N ? (double*)malloc(sizeof(double) * n) : NULL; /* gmres!: p = N V_k, and N (V y) */
    int vcap = mem;
    double** V = (double**)calloc((size_t)vcap, sizeof(double*));
    for (int i = 0; i < vcap; ++i) V[i] = (double*)malloc(sizeof(double) * n);
    double** Z = flex ? (double**)calloc((size_t)vcap, sizeof(double*)) : NULL; /* fgmres!: Z_k = N V_k */
    if (flex)
        for (int i = 0; i < vcap; ++i) Z[i] = (double*)malloc(sizeof(double) * n);
    int cap = mem;  /* capacity of c, s, z (z has cap entries) and R (cap(cap+1)/2) */
    double* c = (double*)calloc((size_t)cap, sizeof(double));
    double* s = (double*)calloc((size_t)cap, sizeof(double));
    double* z = (double*)calloc((size_t)cap, sizeof(double));
    double* R = (double*)calloc((size_t)cap * (cap + 1) / 2, sizeof(double));

    /* OC_DEVRED: every reduction in the device's order (nk_krylov.cpp gmres) */
    const int dev = dr_on(A->P);
    const double bnorm_dev = OC_DEV_BNORM; /* the caller's ||b||, for this solve only (not an inner GMRES's) */
    OC_DEV_BNORM = 0.0;
    double xnorm_dev = 0.0; /* ||x|| of the last cycle's update (k_update_x partials), the restart's FD step */
    oc_fill(n, x, 0.0);
    oc_copy(n, w, b); /* w = b - A*0 */
    if (M) prec_apply(A, M, r0, w); /* r0 = M w */
    /* device: the Newton loop hands ||F(u)|| over as ||b|| (nk_krylov_opts.b_norm), else k_sumsq + k_finalize;
     * with M, ||M b|| from apply_precond */
    double beta = !dev ? oc_norm(n, r0)
                  : M ? sqrt(dr_prec_norm2(A->P, M, r0))
                  : (bnorm_dev > 0.0 ? bnorm_dev : sqrt(dr_reduce(A->P, DR_RED, r0, NULL, 0)));
    double rNorm = beta;
    PUSH_HIST(rNorm);
    const double eps_ = o->atol + o->rtol * rNorm;
    st->inconsistent = 0; st->breakdown = 0;
    if (beta == 0.0) {
        st->niter = 0; st->solved = 1; st->status = 1;
        goto done;
    }
    {
        int npass = 0;
        int64_t iter = 0, inner_iter = 0;
        if (itmax == 0) itmax = 2 * n;
        int64_t inner_itmax = itmax;
        const double btol = pow(DBL_EPSILON, 0.75);
        int breakdown = 0, inconsistent = 0;
        int solved = rNorm <= eps_;
        int tired = iter >= itmax;
        while (!(solved || tired || breakdown)) {
            int64_t nr = 0;
            memset(c, 0, sizeof(double) * cap); memset(s, 0, sizeof(double) * cap);
            memset(z, 0, sizeof(double) * cap); memset(R, 0, sizeof(double) * (size_t)cap * (cap + 1) / 2);
            if (restart) {
                oc_fill(n, xr, 0.0);
                if (npass >= 1) {
                    op_apply(A, w, x, dev ? xnorm_dev : -1.0);
                    oc_axpby(n, 1.0, b, -1.0, w);
                    if (M) prec_apply(A, M, r0, w);
                }
            }
            /* device: the first cycle keeps beta; a restart's ||b - A x|| is the fused EPI_RESID stencil's */
            if (!dev) beta = oc_norm(n, r0);
            else if (restart && npass >= 1)
                beta = M ? sqrt(dr_prec_norm2(A->P, M, r0)) : sqrt(dr_reduce(A->P, DR_TILES, r0, NULL, 0));
            z[0] = beta;
            /* kdivcopy!(n, V[1], r0, rNorm): Krylov.jl divides by rNorm -- beta on the first pass, after a
             * restart the previous cycle's estimate |zeta|, not the beta just computed */
            oc_divcopy(n, V[0], r0, rNorm);
            npass++;
            inner_iter = 0;
            int inner_tired = 0;
            while (!(solved || inner_tired || breakdown)) {
                inner_iter++;
                const int k = (int)inner_iter;
                if (k + 1 > cap) { /* unrestarted GMRES grows its workspace beyond `memory` */
                    int ncap = cap * 2;
                    c = (double*)xrealloc(c, sizeof(double) * ncap); memset(c + cap, 0, sizeof(double) * (ncap - cap));
                    s = (double*)xrealloc(s, sizeof(double) * ncap); memset(s + cap, 0, sizeof(double) * (ncap - cap));
                    z = (double*)xrealloc(z, sizeof(double) * ncap); memset(z + cap, 0, sizeof(double) * (ncap - cap));
                    size_t oR = (size_t)cap * (cap + 1) / 2, nR = (size_t)ncap * (ncap + 1) / 2;
                    R = (double*)xrealloc(R, sizeof(double) * nR); memset(R + oR, 0, sizeof(double) * (nR - oR));
                    cap = ncap;
                }
                if (N) { /* the FD step's ||N V_k||: apply_precond's reduction on the device */
                    double* zk = flex ? Z[k - 1] : pv;
                    prec_apply(A, N, zk, V[k - 1]);
                    op_apply(A, w, zk, dev && A->mode == OC_JV_FD ? sqrt(dr_prec_norm2(A->P, N, zk)) : -1.0);
                } else {
                    /* ||V_1|| = beta / rNorm (1 on the first cycle, |r0| / |zeta| after a restart) */
                    op_apply(A, w, V[k - 1], k == 1 ? beta / rNorm : 1.0);
                }
                if (M) prec_apply(A, M, q, w);
                double Hbis;
                if (dev) {
                    /* h_1 = <V_1, J V_k> from the Jv stencil's tile partials; then np passes, each handing on
                     * the partials of <V_next, q> (<q, q> after the last): the resident sweep's slot partition
                     * and polling wave, or (one pass, or not resident) k_mgs_pass's chunks + reduce_input */
                    const int np = reorth ? 2 * k : k;
                    double h = dr_reduce(A->P, M ? DR_RED : DR_TILES, V[0], q, 0);  /* with M: k_dot after M */
                    for (int t = 0; t < np; ++t) {
                        const int i = t % k;
                        if (t < k) R[nr + i] = h;
                        else R[nr + i] += h;
                        oc_axpy(n, -h, V[i], q);
                        const double* nxt = t + 1 < np ? V[(t + 1) % k] : q;
                        h = dr_reduce(A->P, DR_PASS, nxt, q, np);
                    }
                    Hbis = sqrt(h);
                } else {
                    for (int i = 1; i <= k; ++i) {
                        R[nr + i - 1] = oc_dot(n, V[i - 1], q);
                        oc_axpy(n, -R[nr + i - 1], V[i - 1], q);
                    }
                    if (reorth) {
                        for (int i = 1; i <= k; ++i) {
                            double htmp = oc_dot(n, V[i - 1], q);
                            R[nr + i - 1] += htmp;
                            oc_axpy(n, -htmp, V[i - 1], q);
                        }
                    }
                    Hbis = oc_norm(n, q);
                }
                for (int i = 1; i <= k - 1; ++i) {
                    double Rtmp = c[i - 1] * R[nr + i - 1] + s[i - 1] * R[nr + i];
                    R[nr + i] = s[i - 1] * R[nr + i - 1] - c[i - 1] * R[nr + i];
                    R[nr + i - 1] = Rtmp;
                }
                oc_sym_givens(R[nr + k - 1], Hbis, &c[k - 1], &s[k - 1], &R[nr + k - 1]);
                double zeta = s[k - 1] * z[k - 1];
                z[k - 1] = c[k - 1] * z[k - 1];
                rNorm = fabs(zeta);
                PUSH_HIST(rNorm);
                nr += k;
                int mach = (rNorm + 1.0 <= 1.0);
                solved = (rNorm <= eps_) || mach;
                breakdown = Hbis <= btol;
                inner_tired = restart ? (inner_iter >= (mem < inner_itmax ? mem : inner_itmax)) : (inner_iter >= inner_itmax);
                if (!(solved || inner_tired || breakdown)) {
                    if (k >= vcap) {
                        int nv = vcap * 2;
                        V = (double**)xrealloc(V, sizeof(double*) * nv);
                        for (int i = vcap; i < nv; ++i) V[i] = (double*)malloc(sizeof(double) * n);
                        if (flex) {
                            Z = (double**)xrealloc(Z, sizeof(double*) * nv);
                            for (int i = vcap; i < nv; ++i) Z[i] = (double*)malloc(sizeof(double) * n);
                        }
                        vcap = nv;
                    }
                    oc_divcopy(n, V[k], q, Hbis);
                    z[k] = zeta; /* cap >= k+1 guaranteed by the growth above */
                }
            }
            /* back substitution R y = z, y stored in z */
            const int kk = (int)inner_iter;
            for (int i = kk; i >= 1; --i) {
                int64_t pos = nr + i - kk;
                for (int j = kk; j >= i + 1; --j) {
                    z[i - 1] = z[i - 1] - R[pos - 1] * z[j - 1];
                    pos = pos - j + 1;
                }
                if (fabs(R[pos - 1]) <= btol) { z[i - 1] = 0.0; inconsistent = 1; }
                else z[i - 1] = z[i - 1] / R[pos - 1];
            }
            for (int i = 1; i <= kk; ++i) oc_axpy(n, z[i - 1], flex ? Z[i - 1] : V[i - 1], xr);
            if (N && !flex) { /* gmres!: xr = N (V y) */
                oc_copy(n, pv, xr);
                prec_apply(A, N, xr, pv);
            }
            if (restart) oc_axpy(n, 1.0, xr, x);
            /* device: ||x|| from the x update's partials (k_update_x over wide_blocks, k_finalize) */
            if (dev && restart && A->mode == OC_JV_FD) /* gmres! with N: k_sumsq after x += N (V y) */
                xnorm_dev = sqrt(dr_reduce(A->P, N && !flex ? DR_RED : DR_WIDE, x, NULL, 0));
            iter += inner_iter;
            inner_itmax = itmax - iter;
            tired = iter >= itmax;
        }
        st->niter = iter;
        st->solved = solved;
        st->inconsistent = inconsistent;
        st->breakdown = breakdown;
        st->status = solved ? 1 : (tired ? 2 : (breakdown ? 3 : 0));
    }
done:
    st->n_matvec = A->n_matvec - nmv0;
    if (hist_len) *hist_len = nh;
    free(w);
    if (M) { free(r0); free(q); }
    if (restart) free(xr);
    for (int i = 0; i < vcap; ++i) free(V[i]);
    if (flex) {
        for (int i = 0; i < vcap; ++i) free(Z[i]);
        free(Z);
    }
    free(pv);
    free(V); free(c); free(s); free(z); free(R);
    return 0;
#undef PUSH_HIST
}

/* ------------------------------------------------------------------ CG (Krylov.jl 0.10 cg!, radius = 0, linesearch = false)
 * Left (= the SPD) preconditioner M: z = M r, gamma = <r, z>, p = z + beta p; M = I: z === r. */
int oc_cg(oc_op* A, const double* b, double* x, const oc_krylov_opts* o, oc_krylov_stats* st,
          double* hist, int64_t hist_cap, int64_t* hist_len) {
    const int64_t n = oc_n(A->P);
    int64_t nh = 0;
    const int64_t nmv0 = A->n_matvec;
#define PUSH_HIST(v) do { if (hist && nh < hist_cap) hist[nh] = (v); nh++; } while (0)
    double* r = (double*)malloc(sizeof(double) * n);
    double* p = (double*)malloc(sizeof(double) * n);
    double* Ap = (double*)malloc(sizeof(double) * n);
    const oc_precond* M = (o->M && o->M->kind != OC_PRECOND_NONE) ? o->M : NULL;
    double* zr = M ? (double*)malloc(sizeof(double) * n) : r;
    oc_fill(n, x, 0.0);
    oc_copy(n, r, b);
    if (M) prec_apply(A, M, zr, r);
    oc_copy(n, p, zr);
    /* OC_DEVRED: <r, r> from k_sumsq / k_cg_update's chunks (<r, z> from k_dot with M), <p, Ap> from the
     * stencil's tiles, ||p|| (the FD step) from k_sumsq (nk_krylov.cpp cg) */
    const int dev = dr_on(A->P);
    OC_DEV_BNORM = 0.0; /* the device CG sums ||b|| itself (and an inner GMRES preconditioner must not take it) */
    double gamma = dev ? dr_reduce(A->P, DR_RED, r, M ? zr : NULL, 0) : oc_dot(n, r, zr);
    double rNorm = sqrt(gamma);
    PUSH_HIST(rNorm);
    st->inconsistent = 0; st->breakdown = 0;
    if (gamma == 0.0) {
        st->niter = 0; st->solved = 1; st->status = 1;
    } else {
        int64_t iter = 0, itmax = o->itmax == 0 ? 2 * n : o->itmax;
        double pNorm2 = gamma;
        const double eps_ = o->atol + o->rtol * rNorm;
        int solved = rNorm <= eps_, tired = iter >= itmax, zero_curvature = 0, inconsistent = 0;
        while (!(solved || tired || zero_curvature)) {
            op_apply(A, Ap, p, dev && A->mode == OC_JV_FD ? sqrt(dr_reduce(A->P, DR_RED, p, NULL, 0)) : -1.0);
            double pAp = dev ? dr_reduce(A->P, DR_TILES, p, Ap, 0) : oc_dot(n, p, Ap);
            if (pAp <= DBL_EPSILON * pNorm2) {
                if (fabs(pAp) <= DBL_EPSILON * pNorm2) { zero_curvature = 1; inconsistent = 1; }
            }
            if (zero_curvature) continue;
            double alpha = gamma / pAp;
            oc_axpy(n, alpha, p, x);
            oc_axpy(n, -alpha, Ap, r);
            if (M) prec_apply(A, M, zr, r);
            double gamma_next = !dev ? oc_dot(n, r, zr)
                                : M ? dr_reduce(A->P, DR_RED, r, zr, 0)  /* k_dot after z = M r */
                                    : dr_reduce(A->P, DR_RED1, r, NULL, 0);  /* (k_cg_update) */
            rNorm = sqrt(gamma_next);
            PUSH_HIST(rNorm);
            int mach = (rNorm + 1.0 <= 1.0);
            solved = (rNorm <= eps_) || mach;
            if (!solved) {
                double beta = gamma_next / gamma;
                pNorm2 = gamma_next + beta * beta * pNorm2;
                gamma = gamma_next;
                oc_axpby(n, 1.0, zr, beta, p);
            }
            iter++;
            tired = iter >= itmax;
        }
        st->niter = iter; st->solved = solved; st->inconsistent = inconsistent;
        st->status = solved ? 1 : (tired ? 2 : (zero_curvature ? 4 : 0));
    }
    st->n_matvec = A->n_matvec - nmv0;
    if (hist_len) *hist_len = nh;
    if (M) free(zr);
    free(r); free(p); free(Ap);
    return 0;
#undef PUSH_HIST
}

/* ------------------------------------------------------------------ forcing (Ariadne.jl:185-217) */
double oc_ew_forcing(double eta_max, double gamma, double eta, double tol, double n_res, double n_res_prior) {
    double eta_res = gamma * (n_res * n_res) / (n_res_prior * n_res_prior);
    double eta_safe;
    /* `F.γ * η^2 <= 1 // 10` compares against the exact rational 1/10: for a double x that is x < 0.1 */
    if (gamma * (eta * eta) < 0.1) eta_safe = fmin(eta_max, eta_res);
    else eta_safe = fmin(eta_max, fmax(eta_res, gamma * (eta * eta)));
    return fmin(eta_max, fmax(eta_safe, 0.5 * tol / n_res));
}

/* ------------------------------------------------------------------ Newton driver (Ariadne.jl:288-372) */
int oc_newton_krylov(const oc_problem* P, double* u, const oc_newton_opts* o, oc_newton_stats* st,
                     double* nres_hist, int64_t hist_cap, int64_t* inner_hist) {
    const int64_t n = oc_n(P);
    double* res = (double*)malloc(sizeof(double) * n);
    double* d = (double*)malloc(sizeof(double) * n);
    double* dinv = (o->precond == OC_PRECOND_JACOBI || o->precond == OC_PRECOND_ILU) ? (double*)malloc(sizeof(double) * n) : NULL;
    double* minv = (o->mprecond == OC_PRECOND_JACOBI || o->mprecond == OC_PRECOND_ILU) ? (double*)malloc(sizeof(double) * n) : NULL;
    oc_op A = {P, o->jv_mode, u, res, 0.0, 0};
    int64_t nres_count = 0;
    /* OC_DEVRED: the device driver's norms in its order -- ||F(u)|| from the residual kernel's tiles
     * (nk_residual_norm), ||u|| from the update fused into the solve's last x update (k_update_x's wide
     * chunks; k_sumsq before the first solve; k_axpy_sumsq where the update is not fused) */
    const int dev = dr_on(P);
    double unorm_dev = 0.0;
    oc_residual(P, res, u);
    nres_count++;
    double n_res = dev ? sqrt(dr_reduce(P, DR_TILES, res, NULL, 0)) : oc_norm(n, res);
    int64_t nh = 0;
    if (nres_hist && nh < hist_cap) nres_hist[nh] = n_res;
    nh++;
    const double tol = o->tol_rel * n_res + o->tol_abs;
    double eta = 0.0;
    if (o->forcing == OC_FORCING_FIXED) eta = o->eta_fixed;
    else if (o->forcing == OC_FORCING_EW) eta = o->eta_max;
    int64_t outer = 0, inner = 0;
    while (n_res > tol && outer <= o->max_niter) {
        oc_krylov_opts ko = o->krylov;
        if (!o->rtol_user) ko.rtol = (o->forcing != OC_FORCING_NONE) ? eta : sqrt(DBL_EPSILON);
        oc_krylov_stats ks;
        memset(&ks, 0, sizeof ks);
        if (o->jv_mode == OC_JV_FD)
            A.unorm = !dev ? oc_norm(n, u) : (unorm_dev > 0.0 ? unorm_dev : sqrt(dr_reduce(P, DR_RED, u, NULL, 0)));
        /* N = factory(J) for this step (Ariadne.jl:318-333 passes N through to krylov_solve!) */
        oc_precond Np = {OC_PRECOND_NONE, o->precond_itmax, NULL, P};
        if (o->precond == OC_PRECOND_JACOBI) {
            oc_jacobian_diag(P, dinv, u, 1);
            Np.kind = OC_PRECOND_DIAG;
            Np.diag = dinv;
        } else if (o->precond == OC_PRECOND_ILU) {
            oc_ilu0_factor(P, u, dinv);
            Np.kind = OC_PRECOND_ILU0;
            Np.diag = dinv;
        } else if (o->precond == OC_PRECOND_GMRES) {
            Np.kind = OC_PRECOND_GMRES;
        }
        ko.N = Np.kind != OC_PRECOND_NONE ? &Np : NULL;
        /* M = M(J) (Ariadne.jl:327-329), the same factories */
        oc_precond Mp = {OC_PRECOND_NONE, o->mprecond_itmax, NULL, P};
        if (o->mprecond == OC_PRECOND_JACOBI) {
            oc_jacobian_diag(P, minv, u, 1);
            Mp.kind = OC_PRECOND_DIAG;
            Mp.diag = minv;
        } else if (o->mprecond == OC_PRECOND_ILU) {
            oc_ilu0_factor(P, u, minv);
            Mp.kind = OC_PRECOND_ILU0;
            Mp.diag = minv;
        } else if (o->mprecond == OC_PRECOND_GMRES) {
            Mp.kind = OC_PRECOND_GMRES;
        }
        ko.M = Mp.kind != OC_PRECOND_NONE ? &Mp : NULL;
        ko.flexible = o->algo == OC_ALGO_FGMRES;
        /* b = copy(res) (Ariadne.jl:338): res is not overwritten by our operator, so pass it directly */
        if (dev) OC_DEV_BNORM = n_res;
        if (o->algo == OC_ALGO_CG) oc_cg(&A, res, d, &ko, &ks, NULL, 0, NULL);
        else oc_gmres(&A, res, d, &ko, &ks, NULL, 0, NULL);
        OC_DEV_BNORM = 0.0;
        oc_axpy(n, -1.0, d, u); /* u .-= 1 .* d */
        /* device: fused into the last cycle's x update (wide chunks); no cycle ran, CG, or gmres! with N
         * (x = N (V y) after the update): k_axpy_sumsq (red_blocks) */
        const int fused = ks.niter > 0 && o->algo != OC_ALGO_CG && !(ko.N && o->algo != OC_ALGO_FGMRES);
        if (dev) unorm_dev = sqrt(dr_reduce(P, fused ? DR_WIDE : DR_RED, u, NULL, 0));
        double n_prior = n_res;
        oc_residual(P, res, u);
        nres_count++;
        n_res = dev ? sqrt(dr_reduce(P, DR_TILES, res, NULL, 0)) : oc_norm(n, res);
        if (isinf(n_res) || isnan(n_res)) break;
        if (o->forcing == OC_FORCING_EW) eta = oc_ew_forcing(o->eta_max, o->gamma, eta, tol, n_res, n_prior);
        outer += 1;
        inner += ks.niter;
        if (nres_hist && nh < hist_cap) nres_hist[nh] = n_res;
        if (inner_hist && nh - 1 < hist_cap) inner_hist[nh - 1] = ks.niter;
        nh++;
    }
    st->outer_iterations = outer;
    st->inner_iterations = inner;
    st->n_res = n_res;
    st->solved = n_res <= tol;
    st->n_matvec = A.n_matvec;
    st->n_residual = nres_count;
    st->tol = tol;
    free(res); free(d); free(dinv); free(minv);
    return 0;
}

/* ------------------------------------------------------------------ entry points used by the Python wrapper */
int oc_krylov_solve(const oc_problem* P, int jv_mode, int algo, const double* u, const double* F0,
                    const double* b, double* x, const oc_krylov_opts* o, oc_krylov_stats* st,
                    double* hist, int64_t hist_cap, int64_t* hist_len) {
    oc_op A = {P, jv_mode, u, F0, 0.0, 0};
    if (jv_mode == OC_JV_FD)  /* device: k_sumsq + k_finalize (nk_krylov_solve without a known ||u||) */
        A.unorm = dr_on(P) ? sqrt(dr_reduce(P, DR_RED, u, NULL, 0)) : oc_norm(oc_n(P), u);
    if (algo == OC_ALGO_CG) return oc_cg(&A, b, x, o, st, hist, hist_cap, hist_len);
    oc_krylov_opts oo = *o;
    oo.flexible = algo == OC_ALGO_FGMRES;
    return oc_gmres(&A, b, x, &oo, st, hist, hist_cap, hist_len);
}

void oc_set_threads(int t) { if (t > 0) omp_set_num_threads(t); }
int oc_get_threads(void) { return omp_get_max_threads(); }

/* the shared exp, exported for tests/test_exp.py (its pinning against mpmath) */
void oc_exp(int64_t n, const double* x, double* y) {
    for (int64_t i = 0; i < n; ++i) y[i] = nk_exp(x[i]);
}
void oc_exp_slow(int64_t n, const double* x, double* y) {
    for (int64_t i = 0; i < n; ++i) y[i] = nkx_exp_slow(x[i]);
}
/* the fast phase alone: exp(x) ~ (zh + zl) 2^m; returns how many inputs the Ziv test sent to the slow phase */
int64_t oc_exp_dd(int64_t n, const double* x, double* zh, double* zl, int32_t* m) {
    int64_t slow = 0;
    for (int64_t i = 0; i < n; ++i) {
        int mm;
        zh[i] = nkx_exp_dd(x[i], &NKX_T[0][0], &zl[i], &mm);
        m[i] = mm;
        double y;
        if (!nkx_exp_fast(x[i], &NKX_T[0][0], &y)) ++slow;
    }
    return slow;
}
