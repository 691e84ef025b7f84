/*
 * nkhip.h -- C ABI of libnkhip.so, the MI355X-native JFNK inner loop.
 *
 * Plain pointers and sizes only (no C++ or torch types).  Every entry point replaces one
 * call the reference makes on its hot path; the reference interface is cited per group.
 * A Julia shim binds these with `ccall`; the Python host mirror in
 * newtonkrylov.jl_amd/ binds them with ctypes.
 *
 * Conventions
 *  - Return value: 0 = ok; < 0 = error (NK_E_*; HIP / RCCL errors are mapped, the message is in
 *    nk_last_error(ctx)).  No C++ exception crosses the ABI.
 *  - All device work of a context runs in stream order on the context's single HIP stream.
 *    Functions that return host scalars (nk_dot, nk_norm, nk_residual_norm, solver stats)
 *    synchronise that stream, as Krylov.jl's kdot/knorm return host scalars.
 *  - Vectors are device pointers to the INTERIOR of a grid function allocated by nk_vec_alloc:
 *    the allocation carries one ghost plane before and after the interior along the slowest
 *    axis (zero = physical Dirichlet boundary; written by the halo exchange when distributed).
 *    BLAS-1 primitives touch the n interior entries only.
 */
#ifndef NKHIP_H
#define NKHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- error codes */
#define NK_OK 0
#define NK_E_HIP (-1)
#define NK_E_ARG (-2)
#define NK_E_NOMEM (-3)
#define NK_E_RCCL (-4)
#define NK_E_STATE (-5)
#define NK_E_USER (-6)     /* a user residual / tangent callback returned non-zero */

/* ---------------------------------------------------------------- problem kinds */
#define NK_BRATU1D 1       /* examples/bratu.jl:14-24  bratu!(res, y, (Δx, λ))                         */
#define NK_BRATU2D 2       /* build-defined 2D generalisation                       */
#define NK_HEAT2D_EULER 3  /* examples/implicit.jl:8-13 G_Euler! ∘ examples/heat_2D.jl:45-62 diffusion! */
#define NK_HEAT3D_EULER 4  /* build-defined 3D generalisation                      */
/* the other implicit schemes of examples/implicit.jl composed with diffusion! */
#define NK_HEAT2D_MIDPOINT 5   /* G_Midpoint!  implicit.jl:17-25 (α = nk_problem.alpha)  */
#define NK_HEAT3D_MIDPOINT 6
#define NK_HEAT2D_TRAPEZOID 7  /* G_Trapezoid! implicit.jl:29-37                         */
#define NK_HEAT3D_TRAPEZOID 8

#define NK_USER1D 16       /* user residual F!(res, u, p) given as callbacks, */
#define NK_USER2D 17       /* on a 1D / 2D / 3D grid (the kind fixes the slab axis, as for the      */
#define NK_USER3D 18       /* built-in kinds)                                                      */

#define NK_BC_ZERO 0       /* bc_zero!, examples/heat_2D.jl:28-38 */
#define NK_BC_PERIODIC 1   /* bc_periodic!, examples/heat_2D.jl:15-26 (heat kinds; every extent >= 3):
                              x / y wrap inside the kernels, the slab axis through the ghost planes
                              (a ring exchange: rank 0's lower neighbour is rank nranks - 1)       */

#define NK_JV_EXACT 0      /* exact JVP == Enzyme Forward in mul!(out, J, v), src/Ariadne.jl:48-57 */
#define NK_JV_FD 1         /* (F(u + eps v) - F(u)) / eps, BASELINE.json north star                */

#define NK_ALGO_GMRES 0    /* krylov_workspace(:gmres, …), src/Ariadne.jl:317-318 */
#define NK_ALGO_CG 1       /* krylov_workspace(:cg, …)    (examples/bratu.jl:59-63) */
#define NK_ALGO_FGMRES 2   /* krylov_workspace(:fgmres, …) (examples/bratu.jl:131-157): flexible right-preconditioned GMRES */

/* Right preconditioner N (Krylov.jl's `N`, ldiv = false: z = N v approximates A^{-1} v), as Krylov.jl
 * 0.10 applies it: NK_ALGO_GMRES multiplies J N V_k and updates x += N (V y) once per cycle;
 * NK_ALGO_FGMRES stores Z_k = N V_k and updates x += Z y (N may change from step to step). */
#define NK_PRECOND_NONE 0
#define NK_PRECOND_DIAG 1  /* z = diag .* v  (e.g. Jacobi: diag = 1 ./ diag(J), nk_jacobian_diag) */
#define NK_PRECOND_USER 2  /* z = apply(data, ctx, z, v), enqueued on nk_ctx_stream(ctx)          */
#define NK_PRECOND_GMRES 3 /* z = gmres(J, v; itmax): the GmresPreconditioner of examples/bratu.jl:139-157
                              (Krylov.jl gmres defaults: memory 20, no restart, atol = rtol = √eps), run
                              in `inner` (an NK_ALGO_GMRES workspace of the problem's grid)              */
#define NK_PRECOND_ILU0 4  /* z = (L U)^-1 v: ILU(0) of J in natural order, the `ilu(collect(J))` of examples/bratu.jl:
                              119-137 on J's own pattern (exact LU for the 1D tridiagonal J); diag = D~ from
                              nk_ilu0_factor.  Distributed: block Jacobi (each slab factored on its own) */
typedef int (*nk_user_precond)(void* data, struct nk_ctx* ctx, double* out, const double* in);
typedef struct nk_precond {
    int32_t kind;          /* NK_PRECOND_*                                   */
    const double* diag;    /* NK_PRECOND_DIAG: device grid function          */
    nk_user_precond apply; /* NK_PRECOND_USER                                */
    void* data;
    struct nk_workspace* inner;  /* NK_PRECOND_GMRES: the inner solve's workspace */
    int32_t itmax;               /* NK_PRECOND_GMRES: its itmax                   */
} nk_precond;

typedef struct nk_ctx nk_ctx;
typedef struct nk_workspace nk_workspace;

/* A user residual (kinds NK_USER1D/2D/3D): any F!(res, u, p) the caller can evaluate on device vectors of
 * the problem's grid -- the plug-in point of newton_krylov!'s residual callback
 * (src/Ariadne.jl:288 `F!`, :302, :349).  The callbacks must enqueue their device work on
 * nk_ctx_stream(ctx) (or finish it before returning) and return 0 on success.  When they run, the
 * ghost planes of u (and v) are current: zero (Dirichlet) or the neighbour slab's plane.
 * F is required; J (the exact tangent, what Enzyme's forward mode gives the reference's mul!) is
 * optional -- without it only NK_JV_FD is available. */
typedef int (*nk_user_residual)(void* data, nk_ctx* ctx, double* res, const double* u);
typedef int (*nk_user_tangent)(void* data, nk_ctx* ctx, double* out, const double* u, const double* v);
typedef struct nk_user_ops {
    nk_user_residual F;
    nk_user_tangent J;   /* optional: out = J(u) v                                   */
    nk_user_tangent JT;  /* optional: out = J(u)^T v (Enzyme reverse mode's mul! on transpose(J)) */
    void* data;
} nk_user_ops;

/* F!(res, u, p) of one problem on this rank's slab.  Dimensions are LOCAL interior extents;
 * spacings are global (h = 1/(N_global + 1)).  x is the fastest axis (the reference's
 * column-major first index). */
typedef struct nk_problem {
    int32_t kind;           /* NK_BRATU1D … NK_HEAT3D_TRAPEZOID, NK_USER1D … NK_USER3D */
    int32_t bc;             /* NK_BC_ZERO / NK_BC_PERIODIC */
    int64_t nx, ny, nz;     /* local interior extents (ny = nz = 1 in 1D, nz = 1 in 2D) */
    double hx, hy, hz;      /* grid spacings */
    double lambda;          /* Bratu λ */
    double a, dt;           /* heat diffusivity and time step Δt */
    const double* un;       /* heat: device interior pointer to u_n (borrowed for the call).  Midpoint /
                               trapezoid read its neighbours too: it must be an nk_vec_alloc grid function
                               (its ghost planes are exchanged / wrapped by the library) */
    const nk_user_ops* user;  /* NK_USER*: the callbacks (borrowed for the call) */
    double alpha;           /* NK_HEAT*_MIDPOINT: G_Midpoint!'s α (the reference's default is 0.5) */
} nk_problem;

/* ---------------------------------------------------------------- context / memory */
int nk_device_count(int* count);
int nk_ctx_create(int device, nk_ctx** out);
int nk_ctx_destroy(nk_ctx* ctx);
const char* nk_last_error(nk_ctx* ctx);
int nk_sync(nk_ctx* ctx);
/* the context's HIP stream (hipStream_t): every library kernel and every user callback's work runs on it */
void* nk_ctx_stream(nk_ctx* ctx);

/* similar(u) / zero(u) for a grid function of `p`'s local grid: zero-filled incl. ghost planes. */
int nk_vec_alloc(nk_ctx* ctx, const nk_problem* p, double** out);
int nk_vec_free(nk_ctx* ctx, double* v);
int nk_memcpy_h2d(nk_ctx* ctx, double* dst, const double* src, int64_t n);
int nk_memcpy_d2h(nk_ctx* ctx, double* dst, const double* src, int64_t n);

/* ---------------------------------------------------------------- residual and Jacobian operator */
/* F!(res, u, p): Ariadne calls it at src/Ariadne.jl:302 and :349. */
int nk_residual(nk_ctx* ctx, const nk_problem* p, double* res, const double* u);
/* F!(res, u, p); n_res = norm(res)  fused into one pass (src/Ariadne.jl:302-303, :349-350). */
int nk_residual_norm(nk_ctx* ctx, const nk_problem* p, double* res, const double* u, double* n_res);
/* mul!(out, J::JacobianOperator, v) (src/Ariadne.jl:48-57).  mode NK_JV_EXACT: the tangent of F!
 * (u, v read; F0 unused).  NK_JV_FD: (F(u + eps v) - F0)/eps with F0 = F(u); eps <= 0 selects
 * eps = sqrt(eps_mach) * max(1, ||u||) / ||v||.  Unlike Enzyme, `res` is not rewritten. */
int nk_jv(nk_ctx* ctx, const nk_problem* p, double* out, const double* u, const double* v,
          const double* F0, int32_t mode, double eps);

/* diag(J(u)) of a built-in residual, bit-identical to the diagonal of collect(J) (the tangent
 * kernel's arithmetic on a unit vector); reciprocal = 1 gives 1 ./ diag(J), the Jacobi preconditioner. */
int nk_jacobian_diag(nk_ctx* ctx, const nk_problem* p, double* out, const double* u, int32_t reciprocal);

/* ILU(0) factor of J(u) for NK_PRECOND_ILU0: dtilde (a grid function) receives the pivots D~ of
 * L = I + L_J D~^-1, U = D~ + U_J (J's off-diagonals are constant per axis for the built-in kinds).
 * bc_zero! only. */
int nk_ilu0_factor(nk_ctx* ctx, const nk_problem* p, const double* u, double* dtilde);

/* mul!(out, transpose(J), v) (src/Ariadne.jl:87-107, Enzyme reverse mode): out = J(u)^T v.  The
 * built-in residuals have symmetric Jacobians (3/5/7-point Laplacian plus a diagonal), so this is
 * the exact tangent kernel; user problems need user->JT. */
int nk_jtv(nk_ctx* ctx, const nk_problem* p, double* out, const double* u, const double* v);

/* Batched products: mul!(Out::AbstractMatrix, J, V) (src/Ariadne.jl:67-84, Enzyme BatchDuplicated)
 * and mul!(Out, transpose(J), V) (:109-138).  out[b] = J(u) v[b] for b < k (host arrays of k device
 * grid functions).  One launch per 8 columns reads u, F0 (and u_n) once for all of them; each product
 * is bit-identical to nk_jv / nk_jtv of that column (FD: eps <= 0 picks each column's own step as
 * nk_jv does).  User residuals: one nk_jv / nk_jtv per column. */
int nk_jv_batched(nk_ctx* ctx, const nk_problem* p, int32_t k, double* const* out, const double* u,
                  const double* const* v, const double* F0, int32_t mode, double eps);
int nk_jtv_batched(nk_ctx* ctx, const nk_problem* p, int32_t k, double* const* out, const double* u,
                   const double* const* v);

/* collect(J) / collect(transpose(J)) (src/Ariadne.jl:140-162): the exact Jacobian J(u) as the CSC
 * arrays of the reference's SparseMatrixCSC, 0-based (colptr: n + 1 entries; rowval / nzval: nnz),
 * entries that are exactly 0 dropped as the reference drops them.  Built-in stencils: 2 dim + 1
 * coloured probes in one batched launch + device assembly (values identical to unit probing); user
 * residuals and periodic grids whose extents the colouring does not fit: unit probes (n <= 8192).
 * cap = capacity of rowval / nzval ((2 dim + 1) n always suffices); if nnz > cap, NK_E_ARG with *nnz
 * set.  One rank only. */
int nk_jacobian_collect(nk_ctx* ctx, const nk_problem* p, const double* u, int32_t transpose, int64_t* colptr,
                        int64_t* rowval, double* nzval, int64_t cap, int64_t* nnz);

/* ---------------------------------------------------------------- Krylov vector primitives
 * Krylov.kdot/knorm/kscal!/kaxpy!/kaxpby!/kcopy!/kfill!/kdivcopy!/kref! -- the overload points
 * examples/halovector.jl:51-147 demonstrates for a custom vector type.  n = interior length. */
int nk_dot(nk_ctx* ctx, int64_t n, const double* x, const double* y, double* out);
int nk_norm(nk_ctx* ctx, int64_t n, const double* x, double* out);
int nk_scal(nk_ctx* ctx, int64_t n, double s, double* x);                              /* x = s x       */
int nk_axpy(nk_ctx* ctx, int64_t n, double s, const double* x, double* y);             /* y = s x + y   */
int nk_axpby(nk_ctx* ctx, int64_t n, double s, const double* x, double t, double* y);  /* y = s x + t y */
int nk_copy(nk_ctx* ctx, int64_t n, double* y, const double* x);                       /* y = x         */
/* y = s x + y and ||y|| in one pass: the Newton update u .-= d (src/Ariadne.jl:344) together with the
 * ||u|| the next FD operator needs (nk_krylov_opts.u_norm). */
int nk_axpy_norm(nk_ctx* ctx, int64_t n, double s, const double* x, double* y, double* ynorm);
int nk_fill(nk_ctx* ctx, int64_t n, double* x, double v);                              /* x .= v        */
int nk_divcopy(nk_ctx* ctx, int64_t n, double* y, const double* x, double s);          /* y = x / s     */
int nk_ref(nk_ctx* ctx, int64_t n, double* x, double* y, double c, double s);          /* Givens        */
/* y = exp.(x), correctly rounded: the exp of the Bratu stencils (bratu.jl:21), for user residuals
 * (test/runtests.jl:4-13's exp(x1 - 1)); the CPU oracle compiles the same source (nk_exp.h). */
int nk_vexp(nk_ctx* ctx, int64_t n, double* y, const double* x);

/* One modified-Gram-Schmidt sweep (Krylov.jl gmres! inner loop), fused
 * as the device GMRES runs it: for i = 1..k  h_i = <V_i, q>; q -= h_i V_i  (reorth: a second sweep
 * whose coefficients are added), then h_{k+1} = ||q||.  V: host array of k device pointers; h (host,
 * k + 1 doubles) receives the Hessenberg column.  Synchronises. */
int nk_mgs_step(nk_ctx* ctx, int64_t n, const double* const* V, int32_t k, double* q, int32_t reorth, double* h);

/* ---------------------------------------------------------------- device-resident Krylov solves
 * krylov_workspace(algo, KrylovConstructor(res)) + krylov_solve!(workspace, J, b; kwargs...)
 * (src/Ariadne.jl:317-318, :338), restating Krylov.jl 0.10 gmres!/cg! with M = N = I.  The
 * Arnoldi basis, Hessenberg column and every reduction stay on the device; the host syncs once
 * per Arnoldi step (Givens update + stopping test), not once per kdot. */
typedef struct nk_krylov_opts {
    int32_t restart;              /* gmres: restart = true  (Krylov kwarg)            */
    int32_t reorthogonalization;  /* gmres: double MGS      (heat_2D.jl:131)          */
    int32_t itmax;                /* 0 => 2n                                          */
    int32_t jv_mode;              /* NK_JV_EXACT / NK_JV_FD                           */
    double atol, rtol;            /* Krylov stopping: ||r|| <= atol + rtol ||b||      */
    double b_norm;                /* > 0: ||b|| is known (the Newton loop just computed ||F(u)||): not recomputed */
    double u_norm;                /* > 0: ||u|| is known (FD step size): not recomputed                          */
    double* u_update;             /* non-null: the Newton update u .-= x is fused into the solve's last pass;
                                     x is then NOT stored and stats.u_norm = ||u|| afterwards                */
    const nk_precond* N;          /* right preconditioner (null: none)                                      */
    const nk_precond* M;          /* left preconditioner (null: none): Krylov.jl's `M` (ldiv = false), the
                                     `M = M(J)` Ariadne forwards (src/Ariadne.jl:327-329).  gmres!/fgmres!:
                                     r0 = M (b - A x), q = M A N V_k, the stopping test on ||M r||;
                                     cg!: the SPD preconditioner (z = M r, gamma = <r, z>)                   */
    int32_t f0_is_residual;       /* 1: F0 is exactly F(u) as nk_residual / nk_residual_norm computed it for this
                                     u and problem (the Newton loop's res): the 2D FD operator recomputes F(u)
                                     from the u it loads anyway instead of reading F0 -- bit-identical, 8 B/pt
                                     less traffic.  0 (the default): F0 is read                           */
} nk_krylov_opts;

typedef struct nk_krylov_stats {
    int64_t niter;                /* workspace.stats.niter (Arnoldi / CG iterations)  */
    int32_t solved, inconsistent, breakdown, status; /* status 1 solved 2 tired 3 breakdown 4 zero curvature */
    int64_t n_matvec;             /* mul!(J) calls incl. restart residuals            */
    double u_norm;                /* ||u|| after the fused update (opts.u_update)     */
} nk_krylov_stats;

/* z = N v: Krylov.jl's mulorldiv!(z, N, v, ldiv) for one preconditioner (u, F0, jv_mode: the operator a
 * GMRES preconditioner solves with; unused otherwise).  Synchronises. */
int nk_precond_apply(nk_ctx* ctx, const nk_problem* p, const nk_precond* N, const double* u, const double* F0,
                     int32_t jv_mode, double* z, const double* v);

/* memory = Krylov workspace memory (GMRES restart length; default 20 like Krylov.jl). */
int nk_workspace_create(nk_ctx* ctx, int32_t algo, const nk_problem* p, int32_t memory, nk_workspace** out);
int nk_workspace_destroy(nk_workspace* ws);
double* nk_workspace_x(nk_workspace* ws);  /* workspace.x (device interior pointer) */
/* workspace.V[i + 1] (0-based i) of the last Arnoldi cycle, or null past the allocated basis: the
 * orthonormal basis the last solve built (Krylov.jl keeps it in the workspace too) */
double* nk_workspace_basis(nk_workspace* ws, int32_t i);
/* Solve J(u) x = b; F0 = F(u) (FD mode only).  hist (optional, host) receives the residual-norm
 * estimates (Krylov `history`); *hist_len the number produced (may exceed hist_cap). */
int nk_krylov_solve(nk_workspace* ws, const nk_problem* p, const double* u, const double* F0, const double* b,
                    const nk_krylov_opts* opts, nk_krylov_stats* stats, double* hist, int64_t hist_cap,
                    int64_t* hist_len);

/* ---------------------------------------------------------------- the Newton driver
 * newton_krylov!(F!, u, p, res; kwargs...) (src/Ariadne.jl:288-372) for C / C++ callers: the same
 * loop the Julia and Python hosts run, on top of the calls above.  u is updated in place, res
 * holds F(u) on return. */
#define NK_FORCING_NONE 0   /* forcing = nothing: Krylov's own rtol                        */
#define NK_FORCING_FIXED 1  /* Fixed(η), src/Ariadne.jl:185-192                             */
#define NK_FORCING_EW 2     /* EisenstatWalker(η_max, γ), src/Ariadne.jl:197-217 (default)  */
typedef struct nk_newton_opts {
    double tol_rel, tol_abs;      /* 1e-6, 1e-12: tol = tol_rel ||F(u0)|| + tol_abs            */
    int32_t max_niter;            /* 50 (the loop runs while outer <= max_niter, :336)         */
    int32_t forcing;              /* NK_FORCING_*                                              */
    double eta;                   /* Fixed η (0.1)                                             */
    double eta_max, gamma;        /* EisenstatWalker (0.999, 0.9)                              */
    int32_t algo;                 /* NK_ALGO_GMRES / NK_ALGO_CG                                */
    int32_t memory;               /* Krylov workspace memory (20)                              */
    nk_krylov_opts krylov;        /* krylov_kwargs; jv_mode selects the operator               */
    int32_t rtol_user;            /* krylov.rtol came from krylov_kwargs: it wins (:330-333)   */
} nk_newton_opts;
typedef struct nk_newton_stats {
    int64_t outer_iterations, inner_iterations;  /* Stats (src/Ariadne.jl:265-276)            */
    double n_res, tol;
    int32_t solved;               /* n_res <= tol (:370)                                       */
    int64_t n_matvec, n_residual; /* mul!(J) and F! evaluations                                */
} nk_newton_stats;
int nk_newton_defaults(nk_newton_opts* opts);
/* nres_hist (optional, host): ||F|| after every Newton step, starting with ||F(u0)||. */
int nk_newton_krylov(nk_ctx* ctx, const nk_problem* p, double* u, double* res, const nk_newton_opts* opts,
                     nk_newton_stats* stats, double* nres_hist, int64_t hist_cap, int64_t* hist_len);

/* ---------------------------------------------------------------- multi-GPU (one process per GPU)
 * Slab decomposition along the slowest axis; rank r's lower/upper neighbours are r-1 / r+1.
 * After nk_dist_init every residual / Jv exchanges ghost planes (RCCL send/recv over xGMI) and
 * every dot / norm is all-reduced (RCCL). */
int nk_dist_unique_id(char out[128]);
int nk_dist_init(nk_ctx* ctx, int32_t rank, int32_t nranks, const char id[128]);
int nk_dist_allreduce_sum(nk_ctx* ctx, double* dev_buf, int64_t count);
int nk_halo_exchange(nk_ctx* ctx, const nk_problem* p, double* v);
/* The one-shot peer all-reduce nk_dist_init sets up by itself (NK_DIST_MAILBOX=0 turns it off):
 * every reduction scalar goes from the producing kernel straight into each rank's mailbox
 * (fine-grained memory, IPC-mapped over xGMI) -- no collective launch per inner product.  For
 * callers that exchange the 64-byte IPC handles themselves (no RCCL communicator: reductions only). */
int nk_dist_mailbox_handle(nk_ctx* ctx, char out[64]);
int nk_dist_mailbox_open(nk_ctx* ctx, int32_t rank, int32_t nranks, const char* handles /* nranks x 64 */);
int nk_dist_mailbox_active(nk_ctx* ctx);  /* 1: reductions use the peer mailbox, 0: RCCL / single rank */
/* The process grid of 3D problems (BASELINE config 5: 2 x 2 x 2 blocks): px * py * pz = nranks, rank =
 * (iz py + iy) px + ix, every rank owning an nx x ny x nz block (global spacings, as for slabs).  The
 * default px = py = 1 is the slab decomposition along z.  With px * py > 1 every 3D grid function carries
 * x / y ghost faces besides its z ghost planes, exchanged with the six neighbours through the peer mailbox
 * (packed faces, one launch); call it before allocating vectors.  bc_zero!, built-in residuals; 2D / 1D
 * problems keep slabs.  The reference has no distributed path (examples/halovector.jl:1-45's ghost layer,
 * on every side). */
int nk_dist_grid(nk_ctx* ctx, int32_t px, int32_t py, int32_t pz);
/* Which distributed path this context runs (diagnostics: bench.py prints it for every rank, so a
 * multi-GPU run names the transport it actually used).  No reference counterpart: the reference
 * has no distributed path (its ghost-cell pattern is examples/halovector.jl:1-45). */
typedef struct nk_path_info {
    int32_t rank, nranks, device;
    int32_t ranks_on_device;  /* ranks sharing this GPU, this one included (1: one GPU per rank)        */
    int32_t rccl;             /* an RCCL communicator exists (bootstrap; fallback transport)            */
    int32_t mailbox;          /* reductions and ghost planes through the peer mailbox: 1 device memory
                                 over xGMI (IPC), 2 host shared memory (a peer's device invisible here,
                                 or NK_DIST_MAILBOX=host; planes beyond its small inbox take RCCL)     */
    int32_t resident_sweep;   /* the one-launch resident MGS sweep RAN (sweeps_resident > 0)            */
    int32_t resident_blocks;  /* its grid once set up (0: not run yet)                                 */
    int32_t halo_in_launch;   /* every Krylov Jv that needed v's ghost planes carried them inside the
                                 stencil launch (jv_halo_fused > 0, jv_halo_separate == 0)               */
    int32_t mailbox_error;    /* a mailbox wait timed out (a peer never arrived): sticky                */
    int64_t halo_cap;         /* doubles per IPC inbox plane (larger planes: RCCL send/recv)            */
    char pci_bus_id[32];      /* this rank's device                                                    */
    /* launch counts since the context was created (what the flags above are derived from) */
    int64_t jv_halo_fused;    /* Jv launches with v's ghost planes exchanged inside the launch        */
    int64_t jv_halo_separate; /* Jv launches that exchanged them with a separate launch first        */
    int64_t sweeps_resident;  /* resident MGS sweeps (one launch per Arnoldi step)                     */
    int64_t mgs_passes;       /* per-pass MGS launches (the chain)                                     */
    /* FD operator launches of the built-in stencils, by the instantiation that ran: F(u) recomputed from
       the u rows (F0R: nk_krylov_opts.f0_is_residual) / F0 loaded */
    int64_t jv_fd_f0r;
    int64_t jv_fd_f0_read;
    /* what the exchange costs this rank, measured on the device (wall clock) since the context was created:
       the ghost-plane waits of the slab-end stencil tiles (in-launch) or exchange blocks (separate launch),
       one per tile / block and launch; and the cross-rank reduction waits, one per mailbox all-reduce
       (its consumer's block 0).  Zero without a peer mailbox. */
    int64_t halo_waits;
    int64_t reduce_waits;
    double halo_wait_us;
    double reduce_wait_us;
} nk_path_info;
int nk_dist_path(nk_ctx* ctx, nk_path_info* out);

/* ---------------------------------------------------------------- profiling (HIP events, per kernel class) */
#define NK_PROF_NAME 32
typedef struct nk_prof_entry {
    char name[NK_PROF_NAME];
    int64_t launches;      /* all launches of this kernel class while profiling was on        */
    int64_t timed;         /* launches bracketed by HIP events (every `every`-th one)          */
    double total_ms;       /* sum of the timed launches' event durations                      */
    double bytes;          /* algorithmic bytes (compulsory HBM traffic) of the timed launches */
    double bytes_all;      /* algorithmic bytes of ALL launches (per-launch sizes may vary)   */
    double dram_bytes_all; /* the unique-DRAM model of ALL launches: each distinct operand byte once
                              (re-reads counted as Infinity-Cache hits -- a lower bound on DRAM traffic) */
    char kernel[64];       /* stencil classes: the instantiation the last launch ran, as rocprofv3 names it
                              without the namespace / argument list (e.g. "nk::k_st2d<7, 2, 4, 2, true, true>");
                              empty for the other classes */
} nk_prof_entry;
/* every = 0: off; every = k > 0: time every k-th launch of each kernel class with a pair of HIP
 * events on the context stream (k > 1 keeps the event overhead out of the timed region). */
int nk_prof_enable(nk_ctx* ctx, int32_t every);
int nk_prof_reset(nk_ctx* ctx);
int nk_prof_read(nk_ctx* ctx, nk_prof_entry* out, int32_t cap, int32_t* count);

#ifdef __cplusplus
}
#endif
#endif /* NKHIP_H */
