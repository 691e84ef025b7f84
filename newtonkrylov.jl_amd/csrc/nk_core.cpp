// nk_core.cpp -- context, device memory, profiling and the C-ABI wrappers of the residual,
// Jacobian operator and Krylov vector primitives (include/nkhip.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>

#include "nk_internal.hpp"

namespace nk {

int fail(nk_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

int geometry(nk_ctx* c, const nk_problem* p, Geo* g) {
    if (!p) return fail(c, NK_E_ARG, "null problem");
    if (p->nx < 1 || p->ny < 1 || p->nz < 1) return fail(c, NK_E_ARG, "grid extents must be >= 1");
    switch (p->kind) {
    case NK_BRATU1D:
        if (p->ny != 1 || p->nz != 1) return fail(c, NK_E_ARG, "1D problem needs ny = nz = 1");
        g->dim = 1; g->plane = 1; g->nplanes = p->nx;
        break;
    case NK_BRATU2D:
    case NK_HEAT2D_EULER:
    case NK_HEAT2D_MIDPOINT:
    case NK_HEAT2D_TRAPEZOID:
        if (p->nz != 1) return fail(c, NK_E_ARG, "2D problem needs nz = 1");
        g->dim = 2; g->plane = p->nx; g->nplanes = p->ny;
        break;
    case NK_HEAT3D_EULER:
    case NK_HEAT3D_MIDPOINT:
    case NK_HEAT3D_TRAPEZOID:
        g->dim = 3; g->plane = p->nx * p->ny; g->nplanes = p->nz;
        break;
    case NK_USER1D:
    case NK_USER2D:
    case NK_USER3D:
        if (!p->user || !p->user->F) return fail(c, NK_E_ARG, "user problem needs user->F");
        if (p->kind == NK_USER1D) {
            if (p->ny != 1 || p->nz != 1) return fail(c, NK_E_ARG, "1D problem needs ny = nz = 1");
            g->dim = 1; g->plane = 1; g->nplanes = p->nx;
        } else if (p->kind == NK_USER2D) {
            if (p->nz != 1) return fail(c, NK_E_ARG, "2D problem needs nz = 1");
            g->dim = 2; g->plane = p->nx; g->nplanes = p->ny;
        } else {
            g->dim = 3; g->plane = p->nx * p->ny; g->nplanes = p->nz;
        }
        break;
    default:
        return fail(c, NK_E_ARG, "unknown problem kind");
    }
    if (p->bc == NK_BC_PERIODIC) {
        if (!nk_is_heat(p->kind)) return fail(c, NK_E_ARG, "periodic boundaries are defined for the heat problems (bc_periodic!)");
        // every wrapped axis needs >= 3 points (the slab axis: the whole grid when not distributed)
        if (p->nx < 3 || (g->dim == 3 && p->ny < 3) || (c->nranks <= 1 && g->nplanes < 3))
            return fail(c, NK_E_ARG, "periodic boundaries need >= 3 points along every axis");
    } else if (p->bc != NK_BC_ZERO) {
        return fail(c, NK_E_ARG, "unknown boundary condition");
    }
    if (nk_is_heat(p->kind) && !p->un) return fail(c, NK_E_ARG, "heat problem needs u_n");
    if (g->dim == 3 && c && c->px * c->py > 1) {  // 3D blocks (nk_dist_grid)
        if (p->bc == NK_BC_PERIODIC) return fail(c, NK_E_ARG, "3D blocks: bc_zero! only (periodic problems use z-slabs)");
        if (nk_is_user(p->kind)) return fail(c, NK_E_ARG, "3D blocks: built-in residuals only (user residuals use z-slabs)");
    }
    g->n = p->nx * p->ny * p->nz;
    g->front = (g->plane + 31) / 32 * 32;
    return NK_OK;
}

double* red_slot(nk_ctx* c) {
    double* s = c->red + (size_t)c->red_next * kRedCap;
    c->red_next = (c->red_next + 1) % kRedSlots;
    return s;
}

int mb_check(nk_ctx* c) {
    if (c->mb_err && *(volatile int*)c->mb_err)
        return fail(c, NK_E_RCCL, "peer mailbox: a rank's reduction value or ghost layer never arrived (timeout)");
    if (c->res_err && *(volatile int*)c->res_err) {  // the resident sweep's grid was not co-resident
        *c->res_err = 0;
        c->res_ok = false;  // later solves use one launch per MGS pass
        return fail(c, NK_E_HIP, "resident MGS sweep: a block's partial sum never arrived (timeout); resident sweep disabled");
    }
    if (c->ilu_err && *(volatile int*)c->ilu_err) {  // a strip of the pipelined ILU(0) sweep never advanced
        *c->ilu_err = 0;
        c->ilu_pipe_ok = false;  // later sweeps use the one-work-group level sweep
        c->ilu_redo = true;      // nk_krylov_solve / nk_precond_apply redo their work once on it
        return fail(c, NK_E_HIP, "pipelined ILU(0) sweep: a strip's progress never arrived (timeout); pipelined sweep disabled");
    }
    return NK_OK;
}

int finish_reduction(nk_ctx* c, Red* r) {
    if (r->epoch) {  // the consuming kernel exchanges the per-rank sums through the peer mailbox
        r->len = -(1 + (int)((r->epoch << 15) | (unsigned)r->len));  // = mb_encode (nk_device.hpp)
        r->epoch = 0;
        r->fin = nullptr;
        if (c->res_share > 1) {
            // Ranks sharing this GPU (one-GPU rehearsals): a consumer whose every block spins for the
            // peers' values could hold the CUs a peer's producer needs (two ranks' 512x128x64 GMRES
            // timed out that way).  A one-block k_finalize does the exchange first -- one wave polls,
            // with s_sleep -- and the consumer reads the resolved scalar (len 1: the same bits).
            double* dst = red_slot(c);
            NK_TRY(launch_finalize(c, *r, dst, 0));
            r->ptr = dst;
            r->len = 1;
        }
        return NK_OK;
    }
    if (!c->comm) return NK_OK;
    // collapse this rank's partials to one scalar (normally already done by the producing
    // kernel's last block), then sum the scalars over ranks (RCCL)
    double* dst = r->fin;
    if (!dst) {
        dst = red_slot(c);
        NK_TRY(launch_finalize(c, *r, dst, 0));
    }
    NK_TRY(allreduce_scalar(c, dst, 1));
    r->ptr = dst;
    r->len = 1;
    r->fin = nullptr;
    return NK_OK;
}

// ---------------------------------------------------------------- profiling
int kid(nk_ctx* c, const char* name) {
    auto it = c->kid_of.find(name);
    if (it != c->kid_of.end()) return it->second;
    const int k = (int)c->kid_names.size();
    c->kid_of[name] = k;
    c->kid_names.push_back(name);
    c->acc.emplace_back();
    return k;
}

static int get_event(nk_ctx* c, hipEvent_t* e) {
    if (!c->ev_pool.empty()) {
        *e = c->ev_pool.back();
        c->ev_pool.pop_back();
        return NK_OK;
    }
    NK_HIP(c, hipEventCreate(e));
    return NK_OK;
}

int prof_begin(nk_ctx* c, hipEvent_t* a) {
    NK_TRY(get_event(c, a));
    NK_HIP(c, hipEventRecord(*a, c->stream));
    return NK_OK;
}

int prof_end(nk_ctx* c, int k, hipEvent_t a, double bytes) {
    hipEvent_t b;
    NK_TRY(get_event(c, &b));
    NK_HIP(c, hipEventRecord(b, c->stream));
    c->pending.push_back({k, a, b, bytes});
    if (c->pending.size() > 8192) prof_drain(c, false);
    return NK_OK;
}

void prof_drain(nk_ctx* c, bool blocking) {
    size_t done = 0;
    for (; done < c->pending.size(); ++done) {
        ProfPending& p = c->pending[done];
        if (blocking) {
            (void)hipEventSynchronize(p.b);
        } else if (hipEventQuery(p.b) != hipSuccess) {
            break;
        }
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, p.a, p.b);
        c->acc[p.kid].timed += 1;
        c->acc[p.kid].ms += ms;
        c->acc[p.kid].bytes += p.bytes;
        c->ev_pool.push_back(p.a);
        c->ev_pool.push_back(p.b);
    }
    c->pending.erase(c->pending.begin(), c->pending.begin() + done);
}

}  // namespace nk

using namespace nk;

// =====================================================================================  C ABI
extern "C" {

int nk_device_count(int* count) {
    if (!count) return NK_E_ARG;
    hipError_t e = hipGetDeviceCount(count);
    if (e != hipSuccess) {
        *count = 0;
        return NK_E_HIP;
    }
    return NK_OK;
}

int nk_ctx_create(int device, nk_ctx** out) {
    if (!out) return NK_E_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return NK_E_HIP;
    if (device < 0 || device >= ndev) return NK_E_ARG;
    nk_ctx* c = new nk_ctx();
    c->device = device;
    auto bail = [&](int code) {
        delete c;
        return code;
    };
    if (hipSetDevice(device) != hipSuccess) return bail(NK_E_HIP);
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return bail(NK_E_HIP);
    if (hipMalloc(&c->red, sizeof(double) * (size_t)kRedSlots * kRedCap) != hipSuccess) return bail(NK_E_NOMEM);
    if (hipMalloc(&c->scal, sizeof(double) * kScalCap) != hipSuccess) return bail(NK_E_NOMEM);
    if (hipHostMalloc(&c->hpin, sizeof(double) * kScalCap, hipHostMallocDefault) != hipSuccess) return bail(NK_E_NOMEM);
    if (hipMemset(c->red, 0, sizeof(double) * (size_t)kRedSlots * kRedCap) != hipSuccess) return bail(NK_E_HIP);
    if (hipMemset(c->scal, 0, sizeof(double) * kScalCap) != hipSuccess) return bail(NK_E_HIP);
    *out = c;
    return NK_OK;
}

int nk_dist_free(nk_ctx* ctx);  // nk_dist.cpp

int nk_ctx_destroy(nk_ctx* c) {
    if (!c) return NK_OK;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    nk_dist_free(c);
    for (auto& kv : c->allocs) (void)hipFree(kv.second);
    for (auto& p : c->pending) {
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    (void)hipFree(c->red);
    (void)hipFree(c->scal);
    if (c->tpart) (void)hipFree(c->tpart);
    (void)hipHostFree(c->hpin);
    if (c->res_gran) (void)hipFree(c->res_gran);
    if (c->blk_order) (void)hipFree(c->blk_order);
    if (c->res_err) (void)hipHostFree(c->res_err);
    if (c->ilu_prog) (void)hipFree(c->ilu_prog);
    if (c->ilu_err) (void)hipHostFree(c->ilu_err);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return NK_OK;
}

const char* nk_last_error(nk_ctx* c) { return c ? c->err.c_str() : "null context"; }

void* nk_ctx_stream(nk_ctx* c) { return c ? (void*)c->stream : nullptr; }


int nk_sync(nk_ctx* c) {
    if (!c) return NK_E_ARG;
    NK_HIP(c, hipStreamSynchronize(c->stream));
    if (c->prof) prof_drain(c, false);
    return mb_check(c);
}

int nk_vec_alloc(nk_ctx* c, const nk_problem* p, double** out) {
    if (!c || !out) return NK_E_ARG;
    Geo g;
    NK_TRY(geometry(c, p, &g));
    // start offset: vector j's interior begins (j mod 8) x 128 KB further into its allocation, so that
    // the same index of the fields a kernel streams together (V_i and V_i+1 of an MGS pass; u, v, F0,
    // V_1 of the Jv) does not fall on the same address bits 17-19 (hipMalloc hands out 2 MB-aligned
    // blocks): Bratu 4096^2 +2.1 %, the sweep -2.6 % (profiles/r03/ab_stagger2.log; 256 KB or 1 MB
    // steps gain nothing).  Addresses only: every result is bit-identical.
    static const int stagger = NK_TUNE("NK_ALLOC_STAGGER", 131072);
    static const unsigned smod = (unsigned)std::max(1, NK_TUNE("NK_ALLOC_STAGGER_MOD", 8));
    // (vectors under 2 MB live in sub-allocated pools: no offset, no wasted room)
    const bool big = (size_t)g.n * sizeof(double) >= ((size_t)2 << 20);
    const size_t shift = stagger > 0 && big ? (size_t)(c->alloc_seq++ % smod) * ((size_t)stagger / 256 * 32) : 0;  // doubles
    const int64_t faces = face_words(c, p, g);  // 3D blocks: the x / y ghost faces after the trailing plane
    const size_t total = (size_t)(g.front + g.n + g.plane + faces + 32) + shift;
    void* base = nullptr;
    if (hipMalloc(&base, total * sizeof(double)) != hipSuccess) return fail(c, NK_E_NOMEM, "hipMalloc failed (vector)");
    NK_HIP(c, hipMemsetAsync(base, 0, total * sizeof(double), c->stream));
    NK_HIP(c, hipStreamSynchronize(c->stream));
    double* interior = static_cast<double*>(base) + g.front + shift;
    c->allocs[interior] = base;
    if (faces) c->faced[interior] = faces;
    *out = interior;
    return NK_OK;
}

int nk_vec_free(nk_ctx* c, double* v) {
    if (!c) return NK_E_ARG;
    auto it = c->allocs.find(v);
    if (it == c->allocs.end()) return fail(c, NK_E_ARG, "nk_vec_free: not a vector of this context");
    NK_HIP(c, hipStreamSynchronize(c->stream));
    NK_HIP(c, hipFree(it->second));
    c->faced.erase(v);
    c->allocs.erase(it);
    return NK_OK;
}

int nk_memcpy_h2d(nk_ctx* c, double* dst, const double* src, int64_t n) {
    if (!c || n < 0) return NK_E_ARG;
    NK_HIP(c, hipMemcpyAsync(dst, src, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
    NK_HIP(c, hipStreamSynchronize(c->stream));
    return NK_OK;
}

int nk_memcpy_d2h(nk_ctx* c, double* dst, const double* src, int64_t n) {
    if (!c || n < 0) return NK_E_ARG;
    NK_HIP(c, hipMemcpyAsync(dst, src, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
    NK_HIP(c, hipStreamSynchronize(c->stream));
    return NK_OK;
}

// ---------------------------------------------------------------- residual / Jv
int nk_residual(nk_ctx* c, const nk_problem* p, double* res, const double* u) {
    if (!c || !res || !u) return NK_E_ARG;
    NK_TRY(halo_exchange(c, p, u));
    NK_TRY(exchange_un(c, p));
    StencilIn in{p, MODE_RES, EPI_NONE, res, u, nullptr, nullptr, nullptr, 0.0};
    Red r{};
    return launch_stencil(c, in, &r);
}

int nk_residual_norm(nk_ctx* c, const nk_problem* p, double* res, const double* u, double* n_res) {
    if (!c || !res || !u || !n_res) return NK_E_ARG;
    NK_TRY(halo_exchange(c, p, u));
    NK_TRY(exchange_un(c, p));
    StencilIn in{p, MODE_RES, EPI_SUMSQ, res, u, nullptr, nullptr, nullptr, 0.0};
    Red r{};
    NK_TRY(launch_stencil(c, in, &r));
    NK_TRY(finish_reduction(c, &r));
    NK_TRY(launch_finalize(c, r, c->scal, 1));
    NK_HIP(c, hipMemcpyAsync(c->hpin, c->scal, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    NK_TRY(nk_sync(c));
    *n_res = c->hpin[0];
    return NK_OK;
}

int nk_jv(nk_ctx* c, const nk_problem* p, double* out, const double* u, const double* v, const double* F0, int32_t mode,
          double eps) {
    if (!c || !out || !u || !v) return NK_E_ARG;
    if (mode != NK_JV_EXACT && mode != NK_JV_FD) return fail(c, NK_E_ARG, "bad Jv mode");
    Geo g;
    NK_TRY(geometry(c, p, &g));
    if (mode == NK_JV_FD) {
        if (!F0) return fail(c, NK_E_ARG, "FD Jv needs F0 = F(u)");
        if (eps <= 0.0) {
            double un = 0.0, vn = 0.0;
            NK_TRY(nk_norm(c, g.n, u, &un));
            NK_TRY(nk_norm(c, g.n, v, &vn));
            if (vn == 0.0) return launch_fill(c, g.n, out, 0.0);
            eps = std::sqrt(DBL_EPSILON) * std::fmax(1.0, un) / vn;
        }
    }
    NK_TRY(halo_exchange(c, p, u));
    NK_TRY(exchange_un(c, p));
    StencilIn in{p, mode == NK_JV_FD ? MODE_JFD : MODE_JEXACT, EPI_NONE, out, u, v, F0, nullptr, eps};
    in.xchg_v = true;
    Red r{};
    return launch_stencil(c, in, &r);
}

int nk_jacobian_diag(nk_ctx* c, const nk_problem* p, double* out, const double* u, int32_t reciprocal) {
    if (!c || !out || !u) return NK_E_ARG;
    Geo g;
    NK_TRY(geometry(c, p, &g));
    if (nk_is_user(p->kind)) return fail(c, NK_E_ARG, "diag(J) of a user residual: probe it with collect(J)");
    return launch_jdiag(c, p, out, u, reciprocal);
}

int nk_ilu0_factor(nk_ctx* c, const nk_problem* p, const double* u, double* dtilde) {
    if (!c || !dtilde || !u) return NK_E_ARG;
    Geo g;
    NK_TRY(geometry(c, p, &g));
    if (nk_is_user(p->kind)) return fail(c, NK_E_ARG, "ILU(0) of a user residual: assemble it with collect(J)");
    if (p->bc == NK_BC_PERIODIC) return fail(c, NK_E_ARG, "ILU(0) is implemented for bc_zero! (the wrap breaks the banded pattern)");
    NK_TRY(launch_jdiag(c, p, dtilde, u, 0));
    NK_TRY(launch_ilu0_factor(c, p, g.dim, dtilde));
    // the factor is kept by the preconditioner and reused by later solves: make sure it is whole.  A
    // pipelined sweep that timed out left D~ partly factored -- start again from diag(J) on the level sweep
    const int bad = ilu_pipe_failed(c);
    if (bad < 0) return bad;
    if (bad == 1) {
        NK_TRY(launch_jdiag(c, p, dtilde, u, 0));
        NK_TRY(launch_ilu0_factor(c, p, g.dim, dtilde));
        NK_HIP(c, hipStreamSynchronize(c->stream));
    }
    return NK_OK;
}

int nk_jtv(nk_ctx* c, const nk_problem* p, double* out, const double* u, const double* v) {
    if (!c || !out || !u || !v) return NK_E_ARG;
    Geo g;
    NK_TRY(geometry(c, p, &g));
    if (!nk_is_user(p->kind))  // symmetric Jacobians: J^T v = J v, the exact tangent
        return nk_jv(c, p, out, u, v, nullptr, NK_JV_EXACT, 0.0);
    const nk_user_ops* ops = p->user;
    if (!ops->JT) return fail(c, NK_E_ARG, "transpose product of a user problem needs user->JT");
    NK_TRY(halo_exchange(c, p, u));
    NK_TRY(halo_exchange(c, p, v));
    int rc = 0;
    NK_TRY(launch(c, "user_JT", 0.0, [&] { rc = ops->JT(ops->data, c, out, u, v); }));
    if (rc != 0) return fail(c, NK_E_USER, "user transpose-tangent callback returned " + std::to_string(rc));
    return NK_OK;
}

// ---------------------------------------------------------------- Krylov vector primitives
static int scalar_result(nk_ctx* c, Red r, int sqrt_it, double* out) {
    NK_TRY(finish_reduction(c, &r));
    NK_TRY(launch_finalize(c, r, c->scal, sqrt_it));
    NK_HIP(c, hipMemcpyAsync(c->hpin, c->scal, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    NK_TRY(nk_sync(c));
    *out = c->hpin[0];
    return NK_OK;
}

int nk_dot(nk_ctx* c, int64_t n, const double* x, const double* y, double* out) {
    if (!c || !out || n < 0) return NK_E_ARG;
    Red r{};
    NK_TRY(launch_dot(c, n, x, y, &r));
    return scalar_result(c, r, 0, out);
}

int nk_norm(nk_ctx* c, int64_t n, const double* x, double* out) {
    if (!c || !out || n < 0) return NK_E_ARG;
    Red r{};
    NK_TRY(launch_sumsq(c, n, x, &r));
    return scalar_result(c, r, 1, out);
}

int nk_scal(nk_ctx* c, int64_t n, double s, double* x) { return c ? launch_scal(c, n, s, x) : NK_E_ARG; }
int nk_axpy(nk_ctx* c, int64_t n, double s, const double* x, double* y) { return c ? launch_axpy(c, n, s, x, y) : NK_E_ARG; }
int nk_axpy_norm(nk_ctx* c, int64_t n, double s, const double* x, double* y, double* ynorm) {
    if (!c || !ynorm || n < 0) return NK_E_ARG;
    Red r{};
    NK_TRY(launch_axpy_sumsq(c, n, s, x, y, &r));
    return scalar_result(c, r, 1, ynorm);
}
int nk_axpby(nk_ctx* c, int64_t n, double s, const double* x, double t, double* y) {
    return c ? launch_axpby(c, n, s, x, t, y) : NK_E_ARG;
}
int nk_copy(nk_ctx* c, int64_t n, double* y, const double* x) { return c ? launch_copy(c, n, y, x) : NK_E_ARG; }
int nk_fill(nk_ctx* c, int64_t n, double* x, double v) { return c ? launch_fill(c, n, x, v) : NK_E_ARG; }
int nk_divcopy(nk_ctx* c, int64_t n, double* y, const double* x, double s) { return c ? launch_divcopy(c, n, y, x, s) : NK_E_ARG; }
int nk_ref(nk_ctx* c, int64_t n, double* x, double* y, double cc, double ss) { return c ? launch_ref(c, n, x, y, cc, ss) : NK_E_ARG; }
int nk_vexp(nk_ctx* c, int64_t n, double* y, const double* x) { return c ? (n > 0 ? launch_exp(c, n, y, x) : NK_OK) : NK_E_ARG; }

// One modified-Gram-Schmidt sweep of q against V_1..V_k -- the fused passes the device GMRES runs per
// Arnoldi step, for callers that drive Krylov.jl's loop themselves (SURVEY §8b nk_mgs_step).
int nk_mgs_step(nk_ctx* c, int64_t n, const double* const* V, int32_t k, double* q, int32_t reorth, double* h) {
    if (!c || n < 1 || !V || k < 1 || !q || !h) return NK_E_ARG;
    const int np = reorth ? 2 * k : k;
    if (np + 1 > kScalCap) return fail(c, NK_E_ARG, "nk_mgs_step: k too large for the context's scalar scratch");
    double* col = c->scal;  // device column: h of every pass, then ||q||
    Red red{};
    NK_TRY(launch_dot(c, n, V[0], q, &red));  // partials of <V_1, q>
    for (int t = 0; t < np; ++t) {
        const double* vi = V[t % k];
        const double* vnext = (t + 1 < np) ? V[(t + 1) % k] : nullptr;
        NK_TRY(finish_reduction(c, &red));
        Red nxt{};
        NK_TRY(launch_mgs_pass(c, n, q, vi, vnext, red, col + t, nullptr, &nxt, 0));
        red = nxt;
    }
    NK_TRY(finish_reduction(c, &red));
    NK_TRY(launch_finalize(c, red, col + np, 1));
    NK_HIP(c, hipMemcpyAsync(c->hpin, col, sizeof(double) * (np + 1), hipMemcpyDeviceToHost, c->stream));
    NK_TRY(nk_sync(c));
    NK_TRY(mb_check(c));
    for (int i = 0; i < k; ++i) h[i] = reorth ? c->hpin[i] + c->hpin[k + i] : c->hpin[i];
    h[k] = c->hpin[np];
    return NK_OK;
}

// ---------------------------------------------------------------- profiling
int nk_prof_enable(nk_ctx* c, int32_t every) {
    if (!c || every < 0) return NK_E_ARG;
    if (!every && c->prof) prof_drain(c, true);
    c->prof = every != 0;
    c->prof_every = every > 0 ? every : 1;
    return NK_OK;
}

int nk_prof_reset(nk_ctx* c) {
    if (!c) return NK_E_ARG;
    prof_drain(c, true);
    for (auto& a : c->acc) a = ProfAcc();
    return NK_OK;
}

int nk_prof_read(nk_ctx* c, nk_prof_entry* out, int32_t cap, int32_t* count) {
    if (!c || !count) return NK_E_ARG;
    prof_drain(c, true);
    int m = 0;
    for (size_t k = 0; k < c->kid_names.size(); ++k) {
        if (c->acc[k].launches == 0) continue;
        if (out && m < cap) {
            std::memset(out[m].name, 0, NK_PROF_NAME);
            std::strncpy(out[m].name, c->kid_names[k].c_str(), NK_PROF_NAME - 1);
            out[m].launches = c->acc[k].launches;
            out[m].timed = c->acc[k].timed;
            out[m].total_ms = c->acc[k].ms;
            out[m].bytes = c->acc[k].bytes;
            out[m].bytes_all = c->acc[k].bytes_all;
            out[m].dram_bytes_all = c->acc[k].dram_all;
            std::memset(out[m].kernel, 0, sizeof(out[m].kernel));
            std::strncpy(out[m].kernel, c->acc[k].kernel.c_str(), sizeof(out[m].kernel) - 1);
        }
        ++m;
    }
    *count = m;
    return NK_OK;
}

}  // extern "C"
