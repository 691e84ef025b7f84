// nk_krylov.cpp -- device-resident Krylov.jl 0.10 gmres!/fgmres!/cg! for the Jacobian operator, with
// Krylov.jl's right (N) and left (M) preconditioners.
//
// Restates krylov_workspace(algo, KrylovConstructor(res)) + krylov_solve!(workspace, J, b; kwargs)
// as called by Ariadne (src/Ariadne.jl:317-318, :338, :340, :367) -- SURVEY.md Appendix A.
// Krylov.jl itself is third-party and absent from /root/reference; the same restatement lives in
// oracle/nk_oracle.c (oc_gmres / oc_cg) and the tests check this driver against it.
//
// What moves to the device compared with Krylov.jl's generic loop:
//  * the Arnoldi basis V, q (= w), x, and every reduction;
//  * each Arnoldi step is: one fused Jv kernel (also emits the partials of <V_1, q>), k fused
//    MGS passes (q -= h_i V_i and partials of <V_{i+1}, q>; the last pass emits ||q||^2 partials),
//    one 64-thread finaliser, ONE device->host copy of the Hessenberg column and one sync.
//    Krylov.jl's schedule would sync 2k+1 times (every kdot/knorm returns a host scalar).
//  * the per-cycle kfill!(V[i], 0) of Krylov.jl is dropped: every V[i] read in a cycle is
//    overwritten first, so the zeroing is dead work (no observable difference).
// The Givens rotations, the least-squares back-substitution and all stopping tests run on the
// host on the same scalars, in the same order as Krylov.jl.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "nk_internal.hpp"

struct nk_workspace {
    nk_ctx* c = nullptr;
    int algo = NK_ALGO_GMRES;
    nk_problem prob{};
    int mem = 20;
    int64_t n = 0;
    double* x = nullptr;
    double* w = nullptr;   // gmres: q (= w) of odd steps / restart residual; cg: Ap
    double* w2 = nullptr;  // gmres: q of even steps (the fused Jv reads q_{k-1} while writing q_k)
    double* xr = nullptr;  // gmres restart: Δx (chunked x update);  cg: r
    double* p = nullptr;   // cg: search direction
    std::vector<double*> V;
    std::vector<double*> Z;  // flexible form: Z_k = N V_k (right preconditioner)
    double* mr = nullptr;    // left preconditioner: r0 = M w (gmres) / z = M r (cg)
    double* mw = nullptr;    // left preconditioner: w = A N V_k before q = M w (gmres)
    double* hdev = nullptr;  // device Hessenberg columns: 2 slots of (2*cap + 2) doubles (steps k, k+1 in flight)
    double* ydev = nullptr;  // device y (cap doubles)
    double* bdev = nullptr;  // device divisor of V_1 = r0 / rNorm (fused into step 1)
    bool u_fused = false;    // the last solve applied opts.u_update inside its final x update
    double* hpin = nullptr;  // pinned host mirror of hdev (2 slots), written by the kernels themselves
    double* hpin_dev = nullptr;  // hpin's device address
    double* ypin = nullptr;  // pinned host y
    hipEvent_t col_ready[2] = {nullptr, nullptr};  // Hessenberg column of slot s has landed in hpin
    int cap = 0;             // capacity of hdev / ydev / pinned buffers (in basis vectors)
};

namespace nk {
namespace {

// Grow the Hessenberg/y buffers to hold `need` basis vectors.  Contents are preserved: with the
// one-step-ahead pipeline a column may still be waiting to be read when the basis grows.
int ws_scalars(nk_workspace* ws, int need) {
    if (need <= ws->cap) return NK_OK;
    nk_ctx* c = ws->c;
    int cap = ws->cap ? ws->cap : 64;
    while (cap < need) cap *= 2;
    NK_HIP(c, hipStreamSynchronize(c->stream));
    const size_t ostride = 2 * (size_t)ws->cap + 2, nstride = 2 * (size_t)cap + 2;
    double *hdev = nullptr, *ydev = nullptr, *hpin = nullptr, *ypin = nullptr;
    NK_HIP(c, hipMalloc(&hdev, sizeof(double) * 2 * nstride));
    NK_HIP(c, hipMalloc(&ydev, sizeof(double) * (size_t)cap));
    // fine-grained (coherent) so the kernels' stores are host-visible once the step's event fires
    NK_HIP(c, hipHostMalloc(&hpin, sizeof(double) * 2 * nstride, hipHostMallocMapped | hipHostMallocCoherent));
    NK_HIP(c, hipHostMalloc(&ypin, sizeof(double) * (size_t)cap, hipHostMallocDefault));
    if (ws->cap) {
        for (int slot = 0; slot < 2; ++slot) {
            NK_HIP(c, hipMemcpy(hdev + slot * nstride, ws->hdev + slot * ostride, sizeof(double) * ostride,
                                hipMemcpyDeviceToDevice));
            std::memcpy(hpin + slot * nstride, ws->hpin + slot * ostride, sizeof(double) * ostride);
        }
        (void)hipFree(ws->hdev);
        (void)hipFree(ws->ydev);
        (void)hipHostFree(ws->hpin);
        (void)hipHostFree(ws->ypin);
    }
    ws->hdev = hdev;
    ws->ydev = ydev;
    ws->hpin = hpin;
    ws->ypin = ypin;
    NK_HIP(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&ws->hpin_dev), hpin, 0));
    ws->cap = cap;
    return NK_OK;
}

int ws_basis(nk_workspace* ws, int need) {
    while ((int)ws->V.size() < need) {
        double* v = nullptr;
        NK_TRY(nk_vec_alloc(ws->c, &ws->prob, &v));
        ws->V.push_back(v);
    }
    return NK_OK;
}

// a lazily allocated workspace vector (the left preconditioner's buffers)
int ws_vec(nk_workspace* ws, double** v) {
    if (!*v) NK_TRY(nk_vec_alloc(ws->c, &ws->prob, v));
    return NK_OK;
}

int ws_zbasis(nk_workspace* ws, int need) {
    while ((int)ws->Z.size() < need) {
        double* v = nullptr;
        NK_TRY(nk_vec_alloc(ws->c, &ws->prob, &v));
        ws->Z.push_back(v);
    }
    return NK_OK;
}


inline double sgn(double x) { return (double)((x > 0) - (x < 0)); }

// NK_MGS_RESIDENT=0 (operational) runs one k_mgs_pass launch per MGS pass instead
// of the resident sweep, which needs every CU of the device at once: for a GPU shared with unrelated
// work.  kbench knobs: NK_MGS_ALT=1 alternates the sweep direction of consecutive MGS passes (see
// k_mgs_pass); NK_RES_JV=1 computes the 2D Bratu FD Jv inside the resident sweep's launch (slower,
// DESIGN.md §4)
const int mgs_alt = NK_TUNE("NK_MGS_ALT", 0);
const int mgs_resident = env_cfg("NK_MGS_RESIDENT", 1);
const int mgs_fused_jv = NK_TUNE("NK_RES_JV", 0);

// Krylov.jl sym_givens (real case)
void sym_givens(double a, double b, double* c, double* s, double* rho) {
    if (b == 0.0) {
        *c = (a == 0.0) ? 1.0 : sgn(a);
        *s = 0.0;
        *rho = std::fabs(a);
    } else if (a == 0.0) {
        *c = 0.0;
        *s = sgn(b);
        *rho = std::fabs(b);
    } else if (std::fabs(b) > std::fabs(a)) {
        const double t = a / b;
        *s = sgn(b) / std::sqrt(1.0 + t * t);
        *c = *s * t;
        *rho = b / *s;
    } else {
        const double t = b / a;
        *c = sgn(a) / std::sqrt(1.0 + t * t);
        *s = *c * t;
        *rho = a / *c;
    }
}

// reduce `r` to one host scalar (optionally sqrt) through the context's pinned scratch
int host_scalar(nk_ctx* c, Red r, int sqrt_it, double* out) {
    NK_TRY(finish_reduction(c, &r));
    NK_TRY(launch_finalize(c, r, c->scal, sqrt_it));
    NK_HIP(c, hipMemcpyAsync(c->hpin, c->scal, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    NK_HIP(c, hipStreamSynchronize(c->stream));
    if (c->prof) prof_drain(c, false);
    NK_TRY(mb_check(c));
    *out = c->hpin[0];
    return NK_OK;
}

struct Op;
int gmres(nk_workspace* ws, const nk_problem* p, Op& A, const double* b, const nk_krylov_opts* o, nk_krylov_stats* st,
          double* hist, int64_t hist_cap, int64_t* hist_len);

struct Op {
    nk_ctx* c;
    const nk_problem* p;
    int mode;  // NK_JV_*
    const double* u;
    const double* F0;
    double unorm;
    int64_t n_matvec = 0;
    bool f0r = false;  // F0 is this library's F(u): the 2D FD stencils recompute it instead of loading it

    // out = J v  (+ epilogue).  vnorm: ||v|| for the FD step (1 for Arnoldi basis vectors).
    // With vdiv/vout the operator is applied to v / *vdiv, which is also stored to vout.
    int apply(double* out, const double* v, double vnorm, int epi, const double* aux, Red* red,
              const double* vdiv = nullptr, double* vout = nullptr) {
        ++n_matvec;
        double eps = 0.0;
        if (mode == NK_JV_FD) {
            if (vnorm == 0.0) {  // J 0 = 0
                NK_TRY(launch_fill(c, ws_n(), out, 0.0));
                if (epi == EPI_RESID) NK_TRY(launch_copy(c, ws_n(), out, aux));
                if (epi != EPI_NONE) {
                    if (epi == EPI_DOT) return launch_dot(c, ws_n(), aux, out, red);
                    return launch_sumsq(c, ws_n(), out, red);
                }
                return NK_OK;
            }
            eps = fd_eps(vnorm);
        }
        StencilIn in{p, mode == NK_JV_FD ? MODE_JFD : MODE_JEXACT, epi, out, u, v, F0, aux, eps, vdiv, vout};
        in.xchg_v = true;  // v's ghost planes: exchanged by the stencil launch itself where it can
        in.f0r = f0r;
        return launch_stencil(c, in, red);
    }
    int64_t ws_n() const { return p->nx * p->ny * p->nz; }
    double fd_eps(double vnorm) const { return std::sqrt(DBL_EPSILON) * std::fmax(1.0, unorm) / vnorm; }
};

// z = N v (right preconditioner); *znorm = ||z|| when the FD operator needs it.
//   DIAG   z = d .* v (Jacobi)
//   USER   the caller's device callback
//   GMRES  sol, _ = gmres(J, v; itmax); copyto!(z, sol) -- the GmresPreconditioner of
//          examples/bratu.jl:139-157: Krylov.jl's gmres defaults (memory 20, no restart,
//          atol = rtol = √eps, x0 = 0) on the same operator, in the preconditioner's own workspace
int apply_precond(nk_ctx* c, const nk_problem* p, const nk_precond* N, Op& A, int64_t n, double* z, const double* v,
                  bool need_norm, double* znorm) {
    Red rz{};
    if (N->kind == NK_PRECOND_DIAG) {
        if (!N->diag) return fail(c, NK_E_ARG, "diagonal preconditioner without its diagonal");
        NK_TRY(launch_diag_apply(c, n, z, N->diag, v, need_norm ? &rz : nullptr));
    } else if (N->kind == NK_PRECOND_USER) {
        if (!N->apply) return fail(c, NK_E_ARG, "user preconditioner without its apply callback");
        NK_TRY(halo_exchange(c, p, v));
        int rc = 0;
        NK_TRY(launch(c, "precond_user", 0.0, [&] { rc = N->apply(N->data, c, z, v); }));
        if (rc != 0) return fail(c, NK_E_USER, "user preconditioner callback returned " + std::to_string(rc));
        if (need_norm) NK_TRY(launch_sumsq(c, n, z, &rz));
    } else if (N->kind == NK_PRECOND_ILU0) {
        if (!N->diag) return fail(c, NK_E_ARG, "ILU(0) preconditioner without its factor (nk_ilu0_factor)");
        Geo g;
        NK_TRY(geometry(c, p, &g));
        NK_TRY(launch_ilu0_solve(c, p, g.dim, N->diag, z, v));
        if (need_norm) NK_TRY(launch_sumsq(c, n, z, &rz));
    } else if (N->kind == NK_PRECOND_GMRES) {
        if (!N->inner || N->inner->algo != NK_ALGO_GMRES || N->inner->n != n)
            return fail(c, NK_E_ARG, "GMRES preconditioner needs a GMRES workspace of the problem's size");
        nk_krylov_opts io{};
        io.itmax = N->itmax;
        io.jv_mode = A.mode;
        io.atol = io.rtol = std::sqrt(DBL_EPSILON);
        nk_krylov_stats is{};
        NK_TRY(gmres(N->inner, p, A, v, &io, &is, nullptr, 0, nullptr));
        NK_TRY(launch_copy(c, n, z, N->inner->x));
        if (need_norm) NK_TRY(launch_sumsq(c, n, z, &rz));
    } else {
        return fail(c, NK_E_ARG, "unknown preconditioner kind");
    }
    if (need_norm) NK_TRY(host_scalar(c, rz, 1, znorm));
    return NK_OK;
}

#define PUSH_HIST(v)                                   \
    do {                                               \
        if (hist && nh < hist_cap) hist[nh] = (v);     \
        ++nh;                                          \
    } while (0)

int gmres(nk_workspace* ws, const nk_problem* p, Op& A, const double* b, const nk_krylov_opts* o, nk_krylov_stats* st,
          double* hist, int64_t hist_cap, int64_t* hist_len) {
    nk_ctx* c = ws->c;
    const int64_t n = ws->n;
    const int mem = ws->mem;
    const int restart = o->restart, reorth = o->reorthogonalization;
    int64_t itmax = o->itmax;
    int64_t nh = 0;
    double* x = ws->x;
    double* W[2] = {ws->w, ws->w2};  // q_k lives in W[k & 1]

    // host Krylov state (same layout as Krylov.jl: R column-packed)
    int hcap = mem;
    std::vector<double> cs(hcap), sn(hcap), z(hcap + 1), R((size_t)hcap * (hcap + 1) / 2);

    NK_TRY(ws_basis(ws, mem));
    NK_TRY(ws_scalars(ws, mem + 1));
    // left preconditioner M (ldiv = false): r0 = M (b - A x), q = M A (N V_k); beta and the stopping
    // test measure the preconditioned residual (Krylov.jl 0.10 gmres!)
    const nk_precond* Mp = (o->M && o->M->kind != NK_PRECOND_NONE) ? o->M : nullptr;
    if (Mp) {
        NK_TRY(ws_vec(ws, &ws->mr));
        NK_TRY(ws_vec(ws, &ws->mw));
    }
    // x .= 0 ; r0 = b - A*0 = b.  x is only materialised when no cycle runs: the first cycle's
    // update writes x = Σ y_i V_i directly (bit-identical to 0 + Σ y_i V_i), saving a pass over x.
    Red rb{};
    double beta = o->b_norm;  // the caller may know ||b|| already (Newton: b = F(u), ||F(u)|| just computed)
    const double* r0 = b;
    if (Mp) {  // r0 = M b, beta = ||M b||
        NK_TRY(apply_precond(c, p, Mp, A, n, ws->mr, b, true, &beta));
        r0 = ws->mr;
    } else if (!(beta > 0.0)) {
        NK_TRY(launch_sumsq(c, n, b, &rb));
        NK_TRY(host_scalar(c, rb, 1, &beta));
    }
    double rNorm = beta;
    PUSH_HIST(rNorm);
    const double eps_ = o->atol + o->rtol * rNorm;
    st->inconsistent = 0;
    st->breakdown = 0;
    if (beta == 0.0) {
        NK_TRY(launch_fill(c, n, x, 0.0));
        st->niter = 0;
        st->solved = 1;
        st->status = 1;
        if (hist_len) *hist_len = nh;
        return NK_OK;
    }
    if (itmax == 0) itmax = 2 * n;
    const double btol = std::pow(DBL_EPSILON, 0.75);

    // Issue Arnoldi step k (kernels + async copy of its Hessenberg column) without waiting.
    // Step 1 applies J to the materialised V_1; step k >= 2 applies J to q_{k-1} / h_{k,k-1},
    // reading h from the device and storing V_k on the way (fused kdivcopy!).
    auto slot_dev = [&](int k) { return ws->hdev + (size_t)(k & 1) * (2 * ws->cap + 2); };
    auto slot_pin = [&](int k) { return ws->hpin + (size_t)(k & 1) * (2 * ws->cap + 2); };
    auto slot_pin_dev = [&](int k) { return ws->hpin_dev + (size_t)(k & 1) * (2 * ws->cap + 2); };
    auto npasses_of = [&](int k) { return reorth ? 2 * k : k; };
    const double* v1_src = r0;  // r0 of the current cycle; step 1 applies J to r0 / rNorm and stores V_1
    double v1norm = 1.0;        // ||V_1|| = beta / rNorm
    // right preconditioner, without the one-step-ahead issue (the FD step size needs ||N V_k|| on
    // the host): fgmres! stores Z_k = N V_k and updates x += Z y; gmres! applies N to p = N V_k
    // only for the product and updates x += N (V y) (Krylov.jl 0.10 gmres! / fgmres!)
    const nk_precond* N = (o->N && o->N->kind != NK_PRECOND_NONE) ? o->N : nullptr;
    const bool flex = N && ws->algo == NK_ALGO_FGMRES;
    const bool spec = N == nullptr && Mp == nullptr;
    // vready[k]: step k's resident sweep stored V_{k+1} itself, so step k+1's Jv reads it as is
    std::vector<char> vready(mem + 2, 0);
    auto issue = [&](int k) -> int {
        NK_TRY(ws_basis(ws, k));
        NK_TRY(ws_scalars(ws, k + 1));
        const int np = npasses_of(k);
        double* col = slot_dev(k);
        double* colh = slot_pin_dev(k);  // the kernels mirror every entry into pinned host memory
        double* q = W[k & 1];
        Red red{};
        const double* hprev = k > 1 ? slot_dev(k - 1) + npasses_of(k - 1) : ws->bdev;
        const double* qprev = k > 1 ? W[(k - 1) & 1] : v1_src;
        if ((int)vready.size() < k + 2) vready.resize(k + 2, 0);
        // 2D Bratu, FD Jv, V_k stored by the previous resident sweep: Jv + MGS sweep in ONE launch
        // (q = J V_k is computed into the registers that hold it through the sweep)
        if (mgs_fused_jv && spec && k >= 2 && vready[k - 1] && mgs_resident && A.mode == NK_JV_FD &&
            p->kind == NK_BRATU2D) {
            NK_TRY(ws_basis(ws, k + 1));
            double* vnext = ws->V[k];
            const ResJv jin{A.u, ws->V[k - 1], A.F0, ws->V[0], A.fd_eps(1.0), p->lambda, p->hx * p->hx, p->hy * p->hy, p->nx};
            NK_TRY(halo_exchange(c, p, ws->V[k - 1]));
            const int rc = launch_mgs_sweep(c, n, q, ws->V.data(), k, np, Red{}, col, colh, -1, &vnext, &jin);
            if (rc != NK_OK && rc != 1) return rc;
            if (rc == NK_OK) {
                ++A.n_matvec;
                vready[k] = vnext != nullptr;
                NK_HIP(c, hipEventRecord(ws->col_ready[k & 1], c->stream));
                return NK_OK;
            }
        }
        if (N || Mp) {  // V_k = q_{k-1} / h (r0 / beta), Z_k = N V_k, q = M J Z_k, <V_1, q>
            NK_TRY(launch_fd_point(c, n, nullptr, nullptr, qprev, hprev, 0.0, ws->V[k - 1]));
            const double* zk = ws->V[k - 1];
            double znorm = k == 1 ? v1norm : 1.0;
            if (N) {
                NK_TRY(ws_zbasis(ws, flex ? k : 1));  // gmres!: one p = N V_k buffer; fgmres!: Z_k kept
                double* z = ws->Z[flex ? k - 1 : 0];
                NK_TRY(apply_precond(c, p, N, A, n, z, ws->V[k - 1], A.mode == NK_JV_FD, &znorm));
                zk = z;
            }
            if (Mp) {  // w = J Z_k; q = M w
                NK_TRY(A.apply(ws->mw, zk, znorm, EPI_NONE, nullptr, nullptr));
                double unused = 0.0;
                NK_TRY(apply_precond(c, p, Mp, A, n, q, ws->mw, false, &unused));
                NK_TRY(launch_dot(c, n, ws->V[0], q, &red));
            } else {
                NK_TRY(A.apply(q, zk, znorm, EPI_DOT, ws->V[0], &red));
            }
        } else if (k == 1) {  // fused kdivcopy!(V_1, r0, rNorm) + mul! + <V_1, Jv> (the dot partner is V_1 itself)
            // ||V_1|| = beta / rNorm: 1 on the first cycle, |r0| / |zeta| after a restart (the FD step's ||v||)
            NK_TRY(A.apply(q, v1_src, v1norm, EPI_DOT, nullptr, &red, ws->bdev, ws->V[0]));
        } else if (vready[k - 1]) {  // V_k is in place: mul! + <V_1, Jv> only
            NK_TRY(A.apply(q, ws->V[k - 1], 1.0, EPI_DOT, ws->V[0], &red));
        } else {
            NK_TRY(A.apply(q, qprev, 1.0, EPI_DOT, ws->V[0], &red, hprev, ws->V[k - 1]));
        }
        vready[k] = 0;
        // the whole sweep in one launch with q resident on chip, else one launch per pass
        int rc = 1;
        if (mgs_resident) {
            NK_TRY(finish_reduction(c, &red));
            double* vnext = nullptr;
            if (spec) {  // the speculative path's next Jv can take V_{k+1} from the sweep
                NK_TRY(ws_basis(ws, k + 1));
                vnext = ws->V[k];
            }
            rc = launch_mgs_sweep(c, n, q, ws->V.data(), k, np, red, col, colh, -1, &vnext);
            if (rc != NK_OK && rc != 1) return rc;
            if (rc == NK_OK && vnext) vready[k] = 1;
        }
        if (rc == 1) {
            for (int t = 0; t < np; ++t) {
                const double* vi = ws->V[t % k];
                const double* vnext = (t + 1 < np) ? ws->V[(t + 1) % k] : nullptr;
                NK_TRY(finish_reduction(c, &red));
                Red nxt{};
                NK_TRY(launch_mgs_pass(c, n, q, vi, vnext, red, col + t, colh + t, &nxt, mgs_alt ? (t & 1) : 0));
                red = nxt;
            }
            NK_TRY(finish_reduction(c, &red));
            NK_TRY(launch_finalize(c, red, col + np, 1, colh + np));  // h_{k+1,k} = ||q||
        }
        NK_HIP(c, hipEventRecord(ws->col_ready[k & 1], c->stream));  // column complete in pinned memory
        return NK_OK;
    };

    int npass = 0;
    int64_t iter = 0, inner_iter = 0;
    int64_t inner_itmax = itmax;
    bool breakdown = false, inconsistent = false;
    bool solved = rNorm <= eps_;
    bool tired = iter >= itmax;
    double xnorm = 0.0;  // ||x|| for the FD restart residual (from the fused x update)
    while (!(solved || tired || breakdown)) {
        int64_t nr = 0;
        std::fill(cs.begin(), cs.end(), 0.0);
        std::fill(sn.begin(), sn.end(), 0.0);
        std::fill(z.begin(), z.end(), 0.0);
        std::fill(R.begin(), R.end(), 0.0);
        const double* src = r0;
        if (restart && npass >= 1) {
            Red rr{};
            NK_TRY(A.apply(W[0], x, xnorm, EPI_RESID, b, &rr));  // w = b - A x, fused ||w||^2 partials
            NK_TRY(host_scalar(c, rr, 1, &beta));
            src = W[0];
            if (Mp) {  // r0 = M w, beta = ||r0||
                NK_TRY(apply_precond(c, p, Mp, A, n, ws->mr, W[0], true, &beta));
                src = ws->mr;
            }
        }
        Range cycle_range("gmres_cycle");
        z[0] = beta;
        // kdivcopy!(n, V[1], r0, rNorm) inside step 1's Jv: Krylov.jl divides by rNorm, which is beta on
        // the first pass and, after a restart, the previous cycle's estimate |zeta| (z[1] = beta regardless)
        NK_TRY(launch_fill(c, 1, ws->bdev, rNorm));
        v1_src = src;
        v1norm = beta / rNorm;
        npass++;
        inner_iter = 0;
        bool inner_tired = false;
        NK_TRY(issue(1));
        while (!(solved || inner_tired || breakdown)) {
            inner_iter++;
            const int k = (int)inner_iter;
            if (k + 1 > hcap) {  // unrestarted GMRES grows beyond `memory`
                int nc = hcap * 2;
                cs.resize(nc, 0.0);
                sn.resize(nc, 0.0);
                z.resize(nc + 1, 0.0);
                R.resize((size_t)nc * (nc + 1) / 2, 0.0);
                hcap = nc;
            }
            // speculate: step k+1 unless the cycle certainly ends at k (its kernels only write
            // V_{k+1}, q_{k+1} and slot (k+1)&1, none of which is read if the cycle stops here)
            const bool last = restart ? (inner_iter >= std::min<int64_t>(mem, inner_itmax)) : (inner_iter >= inner_itmax);
            if (!spec && k > 1) NK_TRY(issue(k));  // preconditioned: step k is issued when it is needed
            if (spec && !last) NK_TRY(issue(k + 1));
            NK_HIP(c, hipEventSynchronize(ws->col_ready[k & 1]));
            NK_TRY(mb_check(c));
            if (c->prof) prof_drain(c, false);
            const double* hcol = slot_pin(k);
            const int np = npasses_of(k);
            for (int i = 0; i < k; ++i) R[nr + i] = hcol[i];
            if (reorth)
                for (int i = 0; i < k; ++i) R[nr + i] += hcol[k + i];
            const double Hbis = hcol[np];
            for (int i = 1; i <= k - 1; ++i) {
                const double Rtmp = cs[i - 1] * R[nr + i - 1] + sn[i - 1] * R[nr + i];
                R[nr + i] = sn[i - 1] * R[nr + i - 1] - cs[i - 1] * R[nr + i];
                R[nr + i - 1] = Rtmp;
            }
            sym_givens(R[nr + k - 1], Hbis, &cs[k - 1], &sn[k - 1], &R[nr + k - 1]);
            const double zeta = sn[k - 1] * z[k - 1];
            z[k - 1] = cs[k - 1] * z[k - 1];
            rNorm = std::fabs(zeta);
            PUSH_HIST(rNorm);
            nr += k;
            const bool mach = (rNorm + 1.0 <= 1.0);
            solved = (rNorm <= eps_) || mach;
            breakdown = Hbis <= btol;
            inner_tired = last;
            if (!(solved || inner_tired || breakdown)) z[k] = zeta;  // V_{k+1} = q/h was stored by step k+1
            else if (spec && !last) A.n_matvec -= 1;  // the speculative step k+1 is discarded: not a mul!(J) of the solve
        }
        // back substitution R y = z (Krylov.jl, y stored in z)
        const int kk = (int)inner_iter;
        for (int i = kk; i >= 1; --i) {
            int64_t pos = nr + i - kk;
            for (int j = kk; j >= i + 1; --j) {
                z[i - 1] = z[i - 1] - R[pos - 1] * z[j - 1];
                pos = pos - j + 1;
            }
            if (std::fabs(R[pos - 1]) <= btol) {
                z[i - 1] = 0.0;
                inconsistent = true;
            } else {
                z[i - 1] = z[i - 1] / R[pos - 1];
            }
        }
        NK_TRY(ws_scalars(ws, kk + 1));
        for (int i = 0; i < kk; ++i) ws->ypin[i] = z[i];
        NK_HIP(c, hipMemcpyAsync(ws->ydev, ws->ypin, sizeof(double) * kk, hipMemcpyHostToDevice, c->stream));
        iter += inner_iter;
        inner_itmax = itmax - iter;
        tired = iter >= itmax;
        const bool final_cycle = solved || tired || breakdown;
        const bool need_xnorm = restart && A.mode == NK_JV_FD && !final_cycle;
        double* uu = final_cycle ? o->u_update : nullptr;  // fused Newton update u .-= x
        Red xr{};
        if (N && !flex) {  // gmres!: xr = V y; p = xr; xr = N p; x += xr (restart) -- x = xr otherwise
            uu = nullptr;  // not fused: nk_krylov_solve applies u .-= x afterwards
            NK_TRY(launch_update_x(c, n, W[0], ws->xr, ws->V.data(), kk, ws->ydev, 0, nullptr, nullptr));
            double dummy = 0.0;
            NK_TRY(apply_precond(c, p, N, A, n, ws->Z[0], W[0], false, &dummy));
            if (restart && npass > 1) NK_TRY(launch_axpy(c, n, 1.0, ws->Z[0], x));
            else NK_TRY(launch_copy(c, n, x, ws->Z[0]));
            if (need_xnorm) NK_TRY(launch_sumsq(c, n, x, &xr));
        } else {
            NK_TRY(launch_update_x(c, n, x, ws->xr, N ? ws->Z.data() : ws->V.data(), kk, ws->ydev, restart && npass > 1,
                                   (need_xnorm || uu) ? &xr : nullptr, uu));
        }
        if (uu) {
            NK_TRY(host_scalar(c, xr, 1, &st->u_norm));
            ws->u_fused = true;
        }
        else if (need_xnorm) NK_TRY(host_scalar(c, xr, 1, &xnorm));
        else {
            NK_HIP(c, hipStreamSynchronize(c->stream));  // ypin may be rewritten next cycle
        }
    }
    if (npass == 0) NK_TRY(launch_fill(c, n, x, 0.0));  // solved (or tired) before the first cycle
    st->niter = iter;
    st->solved = solved;
    st->inconsistent = inconsistent;
    st->breakdown = breakdown;
    st->status = solved ? 1 : (tired ? 2 : (breakdown ? 3 : 0));
    if (hist_len) *hist_len = nh;
    return NK_OK;
}

int cg(nk_workspace* ws, Op& A, const double* b, const nk_krylov_opts* o, nk_krylov_stats* st, double* hist,
       int64_t hist_cap, int64_t* hist_len) {
    nk_ctx* c = ws->c;
    const int64_t n = ws->n;
    int64_t nh = 0;
    double *x = ws->x, *r = ws->xr, *p = ws->p, *Ap = ws->w;
    // preconditioner M (Krylov.jl cg!: z = M r, gamma = <r, z>, p = z + beta p); M = I: z === r
    const nk_precond* Mp = (o->M && o->M->kind != NK_PRECOND_NONE) ? o->M : nullptr;
    double* zr = r;
    if (Mp) {
        NK_TRY(ws_vec(ws, &ws->mr));
        zr = ws->mr;
    }
    double unused = 0.0;
    NK_TRY(launch_fill(c, n, x, 0.0));
    NK_TRY(launch_copy(c, n, r, b));
    if (Mp) NK_TRY(apply_precond(c, A.p, Mp, A, n, zr, r, false, &unused));
    NK_TRY(launch_copy(c, n, p, zr));
    Red rg{};
    if (Mp) NK_TRY(launch_dot(c, n, r, zr, &rg));
    else NK_TRY(launch_sumsq(c, n, r, &rg));
    double gamma = 0.0;
    NK_TRY(host_scalar(c, rg, 0, &gamma));
    double rNorm = std::sqrt(gamma);
    PUSH_HIST(rNorm);
    st->inconsistent = 0;
    st->breakdown = 0;
    if (gamma == 0.0) {
        st->niter = 0;
        st->solved = 1;
        st->status = 1;
        if (hist_len) *hist_len = nh;
        return NK_OK;
    }
    int64_t iter = 0, itmax = o->itmax == 0 ? 2 * n : o->itmax;
    double pNorm2 = gamma;
    const double eps_ = o->atol + o->rtol * rNorm;
    bool solved = rNorm <= eps_, tired = iter >= itmax, zero_curvature = false, inconsistent = false;
    while (!(solved || tired || zero_curvature)) {
        double pnorm = 1.0;
        if (A.mode == NK_JV_FD) {
            Red rp{};
            NK_TRY(launch_sumsq(c, n, p, &rp));
            NK_TRY(host_scalar(c, rp, 1, &pnorm));
        }
        Red rpa{};
        NK_TRY(A.apply(Ap, p, pnorm, EPI_DOT, p, &rpa));  // Ap and the partials of <p, Ap>
        double pAp = 0.0;
        NK_TRY(host_scalar(c, rpa, 0, &pAp));
        if (pAp <= DBL_EPSILON * pNorm2) {
            if (std::fabs(pAp) <= DBL_EPSILON * pNorm2) {
                zero_curvature = true;
                inconsistent = true;
            }
        }
        if (zero_curvature) continue;
        const double alpha = gamma / pAp;
        Red rn{};
        NK_TRY(launch_cg_update(c, n, alpha, x, r, p, Ap, &rn));  // x += a p ; r -= a Ap ; <r,r>
        if (Mp) {  // z = M r ; <r, z> (the update's <r,r> partials are not used)
            rn = Red{};
            NK_TRY(apply_precond(c, A.p, Mp, A, n, zr, r, false, &unused));
            NK_TRY(launch_dot(c, n, r, zr, &rn));
        }
        double gamma_next = 0.0;
        NK_TRY(host_scalar(c, rn, 0, &gamma_next));
        rNorm = std::sqrt(gamma_next);
        PUSH_HIST(rNorm);
        const bool mach = (rNorm + 1.0 <= 1.0);
        solved = (rNorm <= eps_) || mach;
        if (!solved) {
            const double beta = gamma_next / gamma;
            pNorm2 = gamma_next + beta * beta * pNorm2;
            gamma = gamma_next;
            NK_TRY(launch_cg_direction(c, n, beta, p, zr));  // p = z + beta p
        }
        iter++;
        tired = iter >= itmax;
    }
    NK_HIP(c, hipStreamSynchronize(c->stream));
    st->niter = iter;
    st->solved = solved;
    st->inconsistent = inconsistent;
    st->status = solved ? 1 : (tired ? 2 : (zero_curvature ? 4 : 0));
    if (hist_len) *hist_len = nh;
    return NK_OK;
}

}  // namespace
}  // namespace nk

using namespace nk;

extern "C" {

int nk_precond_apply(nk_ctx* c, const nk_problem* p, const nk_precond* N, const double* u, const double* F0,
                     int32_t jv_mode, double* z, const double* v) {
    if (!c || !p || !N || !z || !v) return NK_E_ARG;
    Geo g;
    NK_TRY(geometry(c, p, &g));
    if (N->kind == NK_PRECOND_NONE) return launch_copy(c, g.n, z, v);
    if (N->kind == NK_PRECOND_GMRES && (!u || (jv_mode == NK_JV_FD && !F0)))
        return fail(c, NK_E_ARG, "the GMRES preconditioner needs the operator's u (and F0 for FD)");
    Op A{c, p, jv_mode, u, F0, 0.0};
    if (N->kind == NK_PRECOND_GMRES) {
        NK_TRY(halo_exchange(c, p, u));
        NK_TRY(exchange_un(c, p));
        if (jv_mode == NK_JV_FD) {
            Red ru{};
            NK_TRY(launch_sumsq(c, g.n, u, &ru));
            NK_TRY(host_scalar(c, ru, 1, &A.unorm));
        }
    }
    double dummy = 0.0;
    NK_TRY(apply_precond(c, p, N, A, g.n, z, v, false, &dummy));
    int rc = nk_sync(c);
    // a pipelined ILU(0) sweep timed out: once more on the level sweep (one rank only -- with several, the
    // apply recovers by itself, launch_ilu0_solve)
    if (rc != NK_OK && c->ilu_redo && c->nranks == 1) {
        c->ilu_redo = false;
        c->err.clear();
        NK_TRY(apply_precond(c, p, N, A, g.n, z, v, false, &dummy));
        rc = nk_sync(c);
    }
    return rc;
}

int nk_workspace_create(nk_ctx* c, int32_t algo, const nk_problem* p, int32_t memory, nk_workspace** out) {
    if (!c || !p || !out) return NK_E_ARG;
    if (algo != NK_ALGO_GMRES && algo != NK_ALGO_CG && algo != NK_ALGO_FGMRES)
        return fail(c, NK_E_ARG, "unsupported Krylov algorithm");
    Geo g;
    NK_TRY(geometry(c, p, &g));
    nk_workspace* ws = new nk_workspace();
    ws->c = c;
    ws->algo = algo;
    ws->prob = *p;
    ws->prob.un = p->un ? p->un : reinterpret_cast<const double*>(1);  // geometry only
    ws->mem = memory > 0 ? memory : 20;
    ws->n = g.n;
    int rc = NK_OK;
    if ((rc = nk_vec_alloc(c, &ws->prob, &ws->x)) != NK_OK || (rc = nk_vec_alloc(c, &ws->prob, &ws->w)) != NK_OK ||
        (rc = nk_vec_alloc(c, &ws->prob, &ws->xr)) != NK_OK ||
        (algo != NK_ALGO_CG && (rc = nk_vec_alloc(c, &ws->prob, &ws->w2)) != NK_OK) ||
        hipMalloc(&ws->bdev, 2 * sizeof(double)) != hipSuccess ||
        hipEventCreateWithFlags(&ws->col_ready[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ws->col_ready[1], hipEventDisableTiming) != hipSuccess) {
        if (rc == NK_OK) rc = fail(c, NK_E_HIP, "hipEventCreate failed");
        nk_workspace_destroy(ws);
        return rc;
    }
    if (algo == NK_ALGO_CG) {
        if ((rc = nk_vec_alloc(c, &ws->prob, &ws->p)) != NK_OK) {
            nk_workspace_destroy(ws);
            return rc;
        }
    } else {
        if ((rc = ws_basis(ws, ws->mem)) != NK_OK || (rc = ws_scalars(ws, ws->mem + 1)) != NK_OK) {
            nk_workspace_destroy(ws);
            return rc;
        }
    }
    *out = ws;
    return NK_OK;
}

int nk_workspace_destroy(nk_workspace* ws) {
    if (!ws) return NK_OK;
    nk_ctx* c = ws->c;
    for (double* v : ws->V) nk_vec_free(c, v);
    for (double* v : ws->Z) nk_vec_free(c, v);
    for (double* v : {ws->x, ws->w, ws->w2, ws->xr, ws->p, ws->mr, ws->mw})
        if (v) nk_vec_free(c, v);
    for (hipEvent_t e : ws->col_ready)
        if (e) (void)hipEventDestroy(e);
    if (ws->hdev) (void)hipFree(ws->hdev);
    if (ws->ydev) (void)hipFree(ws->ydev);
    if (ws->bdev) (void)hipFree(ws->bdev);
    if (ws->hpin) (void)hipHostFree(ws->hpin);
    if (ws->ypin) (void)hipHostFree(ws->ypin);
    delete ws;
    return NK_OK;
}

double* nk_workspace_x(nk_workspace* ws) { return ws ? ws->x : nullptr; }

double* nk_workspace_basis(nk_workspace* ws, int32_t i) {
    return (ws && i >= 0 && i < (int32_t)ws->V.size()) ? ws->V[(size_t)i] : nullptr;
}

int nk_krylov_solve(nk_workspace* ws, const nk_problem* p, const double* u, const double* F0, const double* b,
                    const nk_krylov_opts* o, nk_krylov_stats* st, double* hist, int64_t hist_cap, int64_t* hist_len) {
    if (!ws || !p || !u || !b || !o || !st) return NK_E_ARG;
    nk_ctx* c = ws->c;
    Geo g;
    NK_TRY(geometry(c, p, &g));
    if (g.n != ws->n) return fail(c, NK_E_ARG, "problem size does not match the workspace");
    if (o->jv_mode == NK_JV_FD && !F0) return fail(c, NK_E_ARG, "FD Jv needs F0 = F(u)");
    *st = nk_krylov_stats{};
    Range solve_range(ws->algo == NK_ALGO_CG ? "cg_solve" : "gmres_solve");
    Op A{c, p, o->jv_mode, u, F0, 0.0};
    A.f0r = o->f0_is_residual != 0 && o->jv_mode == NK_JV_FD;
    NK_TRY(halo_exchange(c, p, u));  // u (and u_n) are constant during the solve: one exchange
    NK_TRY(exchange_un(c, p));
    if (o->jv_mode == NK_JV_FD) {
        A.unorm = o->u_norm;  // known from the fused Newton update (nk_axpy_norm), else one pass
        if (!(A.unorm > 0.0)) {
            Red ru{};
            NK_TRY(launch_sumsq(c, ws->n, u, &ru));
            NK_TRY(host_scalar(c, ru, 1, &A.unorm));
        }
    }
    ws->u_fused = false;
    if (ws->algo == NK_ALGO_CG && o->N && o->N->kind != NK_PRECOND_NONE)
        return fail(c, NK_E_ARG, "the device CG takes no right preconditioner (use GMRES / FGMRES)");
    int rc = (ws->algo == NK_ALGO_CG) ? cg(ws, A, b, o, st, hist, hist_cap, hist_len)
                                      : gmres(ws, p, A, b, o, st, hist, hist_cap, hist_len);
    if (rc != NK_OK && c->ilu_redo && !ws->u_fused && c->nranks == 1) {
        // a pipelined ILU(0) sweep timed out (reported at the step's sync, not by a sync per apply):
        // the whole solve once more, every ILU(0) apply now on the level sweep (u is still untouched).
        // One rank only: a redo on one rank would pair its reductions with its peers' later ones, so a
        // distributed solve checks each apply instead (launch_ilu0_solve)
        c->ilu_redo = false;
        c->err.clear();
        (void)hipStreamSynchronize(c->stream);
        *st = nk_krylov_stats{};
        if (hist_len) *hist_len = 0;
        A.n_matvec = 0;
        rc = (ws->algo == NK_ALGO_CG) ? cg(ws, A, b, o, st, hist, hist_cap, hist_len)
                                      : gmres(ws, p, A, b, o, st, hist, hist_cap, hist_len);
    }
    c->ilu_redo = false;
    st->n_matvec = A.n_matvec;
    if (rc == NK_OK && o->u_update && !ws->u_fused) {  // not fused (CG, early exits): u .-= x, ||u||
        Red ru{};
        NK_TRY(launch_axpy_sumsq(c, ws->n, -1.0, ws->x, o->u_update, &ru));
        NK_TRY(host_scalar(c, ru, 1, &st->u_norm));
    }
    return rc;
}

}  // extern "C"
