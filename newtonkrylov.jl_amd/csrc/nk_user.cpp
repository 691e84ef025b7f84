// nk_user.cpp -- NK_USER1D/2D/3D problems: the residual F!(res, u, p) is the caller's.
//
// The reference's plug-in point is the residual callback of newton_krylov! (src/Ariadne.jl:288,
// called at :302 and :349) together with the operator mul!(out, J, v) (:48-57) that Enzyme
// derives from it.  Here the residual is a host callback that enqueues its own device work on the
// context stream; the library supplies everything around it on the device:
//   * the FD operator  out = (F(u + eps v) - F(u)) / eps: one pass builds w = u + eps v (with the
//     GMRES basis normalisation v = q / h fused in), F(w) is the user's, one pass finishes the
//     quotient together with the reduction the caller asked for (<V1, Jv>, ||.||^2, b - Jv);
//   * the exact operator when the caller also gives the tangent J (Enzyme's forward mode);
//   * ghost planes (zero Dirichlet, or the neighbour slab's plane over RCCL) of every vector the
//     callbacks read, exactly as for the built-in stencils.
// The device GMRES/CG, the Newton driver and all vector primitives are unchanged.
#include <hip/hip_runtime.h>

#include "nk_internal.hpp"

namespace nk {

// FD evaluation point, allocated like any grid function of this geometry and kept on the context
static int user_scratch(nk_ctx* c, const nk_problem* p, const Geo& g, double** w) {
    if (!c->user_w || c->user_w_n != g.n || c->user_w_plane != g.plane) {
        if (c->user_w) NK_TRY(nk_vec_free(c, c->user_w));
        c->user_w = nullptr;
        NK_TRY(nk_vec_alloc(c, p, &c->user_w));
        c->user_w_n = g.n;
        c->user_w_plane = g.plane;
    }
    *w = c->user_w;
    return NK_OK;
}

static int user_call(nk_ctx* c, const char* what, int rc) {
    if (rc != 0) return fail(c, NK_E_USER, std::string("user ") + what + " callback returned " + std::to_string(rc));
    return NK_OK;
}

int launch_user(nk_ctx* c, const StencilIn& in, Red* red) {
    const nk_problem* p = in.p;
    const nk_user_ops* ops = p->user;
    Geo g;
    NK_TRY(geometry(c, p, &g));
    int rc = 0;
    bool fd = false;
    switch (in.mode) {
    case MODE_RES:
        NK_TRY(launch(c, "user_F", 0.0, [&] { rc = ops->F(ops->data, c, in.out, in.u); }));
        NK_TRY(user_call(c, "residual", rc));
        break;
    case MODE_JFD: {
        double* w = nullptr;
        NK_TRY(user_scratch(c, p, g, &w));
        NK_TRY(launch_fd_point(c, g.n, w, in.u, in.v, in.vdiv, in.eps, in.vout));
        NK_TRY(halo_exchange(c, p, w));
        NK_TRY(launch(c, "user_F", 0.0, [&] { rc = ops->F(ops->data, c, in.out, w); }));
        NK_TRY(user_call(c, "residual", rc));
        fd = true;
        break;
    }
    default: {  // MODE_JEXACT
        if (!ops->J) return fail(c, NK_E_ARG, "exact Jv of a user problem needs user->J (or use NK_JV_FD)");
        const double* v = in.v;
        if (in.vdiv && !in.vout) return fail(c, NK_E_ARG, "normalised Jv input needs its output vector");
        if (in.vdiv) {  // materialise V_k = q / h first: the tangent callback reads a plain vector
            NK_TRY(launch_fd_point(c, g.n, nullptr, nullptr, in.v, in.vdiv, 0.0, in.vout));
            NK_TRY(halo_exchange(c, p, in.vout));
            v = in.vout;
        }
        NK_TRY(launch(c, "user_J", 0.0, [&] { rc = ops->J(ops->data, c, in.out, in.u, v); }));
        NK_TRY(user_call(c, "tangent", rc));
        break;
    }
    }
    // dot partner: aux, or (V_1 = r0 / beta fused into the first Jv) the normalised input just stored
    const double* aux = (in.epi == EPI_DOT && !in.aux) ? in.vout : in.aux;
    if (in.epi == EPI_DOT && !aux) return fail(c, NK_E_ARG, "dot epilogue needs its partner");
    if (fd || in.epi != EPI_NONE) NK_TRY(launch_user_epi(c, g.n, fd, in.out, in.F0, in.eps, in.epi, aux, red));
    return NK_OK;
}

}  // namespace nk
