// bratu2d_newton.cpp -- a C++ caller of libnkhip.so through the public C ABI only (include/nkhip.h):
// 2D Bratu on an N x N grid, u0 = sin(pi x) sin(pi y), newton_krylov! with GMRES(memory) and the
// Eisenstat-Walker forcing (src/Ariadne.jl:288-372), FD or exact Jv.  Prints one JSON line.
//
//   bin/bratu2d_newton [N=256] [jv=fd|exact] [memory=30] [restart=1]
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "nkhip.h"

#define CHECK(ctx, call)                                                                  \
    do {                                                                                  \
        int rc_ = (call);                                                                 \
        if (rc_ != NK_OK) {                                                               \
            std::fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, nk_last_error(ctx)); \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)

int main(int argc, char** argv) {
    const int64_t N = argc > 1 ? std::atoll(argv[1]) : 256;
    const bool fd = argc > 2 ? std::strcmp(argv[2], "exact") != 0 : true;
    const int memory = argc > 3 ? std::atoi(argv[3]) : 30;
    const int restart = argc > 4 ? std::atoi(argv[4]) : 1;
    const double h = 1.0 / (double)(N + 1), lambda = 3.51382;  // examples/bratu.jl:41-42

    nk_ctx* ctx = nullptr;
    if (nk_ctx_create(0, &ctx) != NK_OK) {
        std::fprintf(stderr, "no usable GPU\n");
        return 1;
    }
    nk_problem p{};
    p.kind = NK_BRATU2D;
    p.bc = NK_BC_ZERO;
    p.nx = N;
    p.ny = N;
    p.nz = 1;
    p.hx = p.hy = h;
    p.hz = 1.0;
    p.lambda = lambda;
    double *u = nullptr, *res = nullptr;
    CHECK(ctx, nk_vec_alloc(ctx, &p, &u));
    CHECK(ctx, nk_vec_alloc(ctx, &p, &res));
    std::vector<double> host((size_t)(N * N));
    for (int64_t j = 0; j < N; ++j)
        for (int64_t i = 0; i < N; ++i) host[(size_t)(j * N + i)] = std::sin(M_PI * (i + 1) * h) * std::sin(M_PI * (j + 1) * h);
    CHECK(ctx, nk_memcpy_h2d(ctx, u, host.data(), N * N));

    nk_newton_opts o;
    CHECK(ctx, nk_newton_defaults(&o));
    o.memory = memory;
    o.krylov.restart = restart;
    o.krylov.jv_mode = fd ? NK_JV_FD : NK_JV_EXACT;
    nk_newton_stats st;
    double hist[64];
    int64_t nh = 0;
    const auto t0 = std::chrono::steady_clock::now();
    CHECK(ctx, nk_newton_krylov(ctx, &p, u, res, &o, &st, hist, 64, &nh));
    CHECK(ctx, nk_sync(ctx));
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    CHECK(ctx, nk_memcpy_d2h(ctx, host.data(), u, N * N));
    double umax = 0.0;
    for (double v : host) umax = std::fmax(umax, std::fabs(v));
    std::printf("{\"N\": %lld, \"jv\": \"%s\", \"solved\": %s, \"outer\": %lld, \"inner\": %lld, \"n_matvec\": %lld, "
                "\"n_res\": %.17g, \"tol\": %.17g, \"u_max\": %.17g, \"seconds\": %.6f, \"n_res_history\": [",
                (long long)N, fd ? "fd" : "exact", st.solved ? "true" : "false", (long long)st.outer_iterations,
                (long long)st.inner_iterations, (long long)st.n_matvec, st.n_res, st.tol, umax, secs);
    for (int64_t k = 0; k < nh && k < 64; ++k) std::printf("%s%.17g", k ? ", " : "", hist[k]);
    std::printf("]}\n");
    CHECK(ctx, nk_vec_free(ctx, u));
    CHECK(ctx, nk_vec_free(ctx, res));
    nk_ctx_destroy(ctx);
    return 0;
}
