// nk_newton.cpp -- newton_krylov! (src/Ariadne.jl:288-372) as a C-ABI entry point.
//
// The reference's driver is host code; the Julia shim and the Python mirror keep it in their host
// language.  This is the same loop for C / C++ callers, line for line: tol = tol_rel ||F(u0)|| +
// tol_abs (:305), `while n_res > tol && outer <= max_niter` (:336), rtol = η unless the caller's
// krylov_kwargs carry rtol (:323-333), b = F(u) (:338; our operator never rewrites res, so res is
// passed directly), u .-= d (:344), non-finite ||F|| ends the loop (:353-356), the forcing update
// (:357-361) and Stats (:362-367).  Every O(n) step runs in this library on the device.
#include <cfloat>
#include <cmath>
#include <vector>

#include "nk_internal.hpp"

namespace {

// EisenstatWalker, src/Ariadne.jl:207-217 (`γ η² <= 1//10` is an exact rational: `< 0.1` for a double)
double ew_forcing(double eta_max, double gamma, double eta, double tol, double n_res, double n_res_prior) {
    const double eta_res = gamma * (n_res * n_res) / (n_res_prior * n_res_prior);
    double eta_safe;
    if (gamma * (eta * eta) < 0.1) eta_safe = std::fmin(eta_max, eta_res);
    else eta_safe = std::fmin(eta_max, std::fmax(eta_res, gamma * (eta * eta)));
    return std::fmin(eta_max, std::fmax(eta_safe, 0.5 * tol / n_res));
}

}  // namespace

extern "C" {

int nk_newton_defaults(nk_newton_opts* o) {
    if (!o) return NK_E_ARG;
    *o = nk_newton_opts{};
    o->tol_rel = 1e-6;
    o->tol_abs = 1e-12;
    o->max_niter = 50;
    o->forcing = NK_FORCING_EW;
    o->eta = 0.1;
    o->eta_max = 0.999;
    o->gamma = 0.9;
    o->algo = NK_ALGO_GMRES;
    o->memory = 20;
    o->krylov.jv_mode = NK_JV_EXACT;
    o->krylov.atol = std::sqrt(DBL_EPSILON);
    o->krylov.rtol = std::sqrt(DBL_EPSILON);
    return NK_OK;
}

int nk_newton_krylov(nk_ctx* c, const nk_problem* p, double* u, double* res, const nk_newton_opts* o,
                     nk_newton_stats* st, double* nres_hist, int64_t hist_cap, int64_t* hist_len) {
    if (!c || !p || !u || !res || !o || !st) return NK_E_ARG;
    if (o->forcing < NK_FORCING_NONE || o->forcing > NK_FORCING_EW) return nk::fail(c, NK_E_ARG, "bad forcing");
    nk::Geo g;
    NK_TRY(nk::geometry(c, p, &g));
    *st = nk_newton_stats{};
    int64_t nh = 0;
    auto push = [&](double v) {
        if (nres_hist && nh < hist_cap) nres_hist[nh] = v;
        ++nh;
    };
    double n_res = 0.0;
    NK_TRY(nk_residual_norm(c, p, res, u, &n_res));  // F!(res, u, p); n_res = norm(res)  (:302-303)
    st->n_residual = 1;
    push(n_res);
    const double tol = o->tol_rel * n_res + o->tol_abs;
    double eta = o->forcing == NK_FORCING_FIXED ? o->eta : o->eta_max;
    nk_workspace* ws = nullptr;
    NK_TRY(nk_workspace_create(c, o->algo, p, o->memory > 0 ? o->memory : 20, &ws));
    int rc = NK_OK;
    int64_t outer = 0, inner = 0;
    double u_norm = 0.0;  // ||u|| after the fused update (FD step size of the next solve); 0 = unknown
    while (n_res > tol && outer <= o->max_niter) {
        nk::Range step_range("newton_step");
        nk_krylov_opts ko = o->krylov;
        if (!o->rtol_user && o->forcing != NK_FORCING_NONE) ko.rtol = eta;
        ko.b_norm = n_res;  // b = F(u): its norm is the n_res just computed
        ko.u_norm = u_norm;
        ko.u_update = u;    // u .-= d fused into the solve's last pass (d = workspace.x is not stored)
        ko.f0_is_residual = 1;  // res = F(u) was just computed by nk_residual_norm
        nk_krylov_stats ks{};
        const double* F0 = ko.jv_mode == NK_JV_FD ? res : nullptr;
        if ((rc = nk_krylov_solve(ws, p, u, F0, res, &ko, &ks, nullptr, 0, nullptr)) != NK_OK) break;
        st->n_matvec += ks.n_matvec;
        u_norm = ks.u_norm;  // ||u|| after u .-= 1 .* d (:344)
        const double n_prior = n_res;
        if ((rc = nk_residual_norm(c, p, res, u, &n_res)) != NK_OK) break;
        st->n_residual++;
        if (std::isinf(n_res) || std::isnan(n_res)) break;  // "Inner solver blew up" (:353-356)
        if (o->forcing == NK_FORCING_EW) eta = ew_forcing(o->eta_max, o->gamma, eta, tol, n_res, n_prior);
        outer += 1;
        inner += ks.niter;
        push(n_res);
    }
    nk_workspace_destroy(ws);
    st->outer_iterations = outer;
    st->inner_iterations = inner;
    st->n_res = n_res;
    st->tol = tol;
    st->solved = n_res <= tol;
    if (hist_len) *hist_len = nh;
    return rc;
}

}  // extern "C"
