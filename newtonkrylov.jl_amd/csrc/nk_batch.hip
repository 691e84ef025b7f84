// nk_batch.hip -- batched Jacobian-vector products and the device assembly of collect(J).
//
// mul!(Out::AbstractMatrix, J, V) (src/Ariadne.jl:67-84) pushes k tangents through ONE Enzyme
// forward pass (BatchDuplicated).  k_jv_batch is that pass for the built-in stencils: every point
// reads u (and F(u), u_n) once and produces all k products, instead of k launches that re-read
// u / F0 k times (FD: (2 + 2k) instead of 4k words per point).  Every product is bit-identical to
// the single-vector kernel's (same operands, same association order, -ffp-contract=off).
//
// collect(J) (src/Ariadne.jl:140-162) applies J to the n unit vectors.  For the 3/5/7-point
// stencils the n probes collapse into 2 dim + 1 coloured probes (a distance-2 colouring: every
// probe entry is exactly one Jacobian entry, computed from the same operands as the unit-vector
// probe), which k_jv_batch evaluates in one launch; two small kernels and a device scan then write
// the CSC arrays the reference's SparseMatrixCSC holds (zeros dropped, `if out[i] != 0`).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <vector>

#include "nk_exp_dev.hpp"
#include "nk_internal.hpp"

namespace nk {

constexpr int kMaxBatch = 8;  // products per k_jv_batch launch (larger batches run in chunks)

struct BArgs {
    double* out[kMaxBatch];
    const double* v[kMaxBatch];
    double eps[kMaxBatch];
    const double* u;
    const double* F0;
    const double* un;
    int nb;
    int per;  // bc_periodic!: x (and y in 3D) wrap in the kernel, the slab axis through the ghost planes
    int64_t n, nx, ny, nz;
    double hx2, hy2, hz2, lam, a, dt, alpha;
};

namespace {

template <int KIND>
constexpr int kind_dim() {
    return KIND == NK_BRATU1D ? 1 : ((KIND == NK_HEAT3D_EULER || KIND == NK_HEAT3D_MIDPOINT || KIND == NK_HEAT3D_TRAPEZOID) ? 3 : 2);
}
template <int KIND>
constexpr int kind_scheme() {
    return (KIND == NK_HEAT2D_MIDPOINT || KIND == NK_HEAT3D_MIDPOINT)
               ? 1
               : ((KIND == NK_HEAT2D_TRAPEZOID || KIND == NK_HEAT3D_TRAPEZOID) ? 2 : 0);
}
constexpr bool kind_bratu(int k) { return k == NK_BRATU1D || k == NK_BRATU2D; }

// ((p - 2c) + m) / h^2 exactly as the reference writes it (bratu.jl:19, heat_2D.jl:55-58)
__device__ __forceinline__ double lp(double c, double p, double m, double h2) { return ((p - 2.0 * c) + m) / h2; }

// The stencil points of interior point o (the centre first): offsets and existence.  The slow axis
// always exists (ghost planes in memory: zero, the neighbour slab's plane, or the periodic wrap);
// the faster axes are predicated (bc_zero!) or wrap (bc_periodic!).  Order: c, x+, x-, y+, y-, z+, z-.
template <int DIM>
struct Nbrs {
    int64_t off[2 * DIM + 1];
    bool ok[2 * DIM + 1];
};
template <int DIM>
__device__ __forceinline__ Nbrs<DIM> nbrs(const BArgs& B, int64_t o) {
    Nbrs<DIM> s;
    s.off[0] = o;
    s.ok[0] = true;
    if constexpr (DIM == 1) {
        s.off[1] = o + 1; s.ok[1] = true;
        s.off[2] = o - 1; s.ok[2] = true;
    } else {
        const int64_t i = o % B.nx;
        if (B.per) {
            s.off[1] = i + 1 < B.nx ? o + 1 : o - (B.nx - 1); s.ok[1] = true;
            s.off[2] = i >= 1 ? o - 1 : o + (B.nx - 1); s.ok[2] = true;
        } else {
            s.off[1] = o + 1; s.ok[1] = i + 1 < B.nx;
            s.off[2] = o - 1; s.ok[2] = i >= 1;
        }
        if constexpr (DIM == 2) {
            s.off[3] = o + B.nx; s.ok[3] = true;
            s.off[4] = o - B.nx; s.ok[4] = true;
        } else {
            const int64_t pl = B.nx * B.ny;
            const int64_t j = (o / B.nx) % B.ny;
            if (B.per) {
                s.off[3] = j + 1 < B.ny ? o + B.nx : o - (B.ny - 1) * B.nx; s.ok[3] = true;
                s.off[4] = j >= 1 ? o - B.nx : o + (B.ny - 1) * B.nx; s.ok[4] = true;
            } else {
                s.off[3] = o + B.nx; s.ok[3] = j + 1 < B.ny;
                s.off[4] = o - B.nx; s.ok[4] = j >= 1;
            }
            s.off[5] = o + pl; s.ok[5] = true;
            s.off[6] = o - pl; s.ok[6] = true;
        }
    }
    return s;
}

// Laplacian sum of the stencil field f[] in the single-vector kernels' association order
template <int DIM>
__device__ __forceinline__ double lsum_of(const BArgs& B, const double* f) {
    if constexpr (DIM == 1) return lp(f[0], f[1], f[2], B.hx2);
    if constexpr (DIM == 2) return lp(f[0], f[1], f[2], B.hx2) + lp(f[0], f[3], f[4], B.hy2);
    return (lp(f[0], f[1], f[2], B.hx2) + lp(f[0], f[3], f[4], B.hy2)) + lp(f[0], f[5], f[6], B.hz2);
}

// All nb products at the point o: u, F0, u_n (and their stencil values) are loaded once.
template <int KIND, int MODE>
__global__ __launch_bounds__(kBlock) void k_jv_batch(BArgs B) {
    constexpr int DIM = kind_dim<KIND>(), NP = 2 * DIM + 1, SCH = kind_scheme<KIND>();
    constexpr bool FD = MODE == MODE_JFD;
    for (int64_t o = (int64_t)blockIdx.x * kBlock + threadIdx.x; o < B.n; o += (int64_t)gridDim.x * kBlock) {
        const Nbrs<DIM> s = nbrs<DIM>(B, o);
        double uu[NP], gg[NP];  // u (FD) and u_n (midpoint / trapezoid FD) at the stencil points
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            uu[q] = (FD && s.ok[q]) ? B.u[s.off[q]] : 0.0;
            gg[q] = (FD && SCH != 0 && s.ok[q]) ? B.un[s.off[q]] : 0.0;
        }
        const double eu = (!FD && kind_bratu(KIND)) ? nk_exp(B.u[o]) : 0.0;       // Enzyme tangent of λ exp(u)
        const double unc = (FD && !kind_bratu(KIND)) ? B.un[o] : 0.0;
        const double f0 = FD ? B.F0[o] : 0.0;
        const double lsumg = (FD && SCH == 2) ? lsum_of<DIM>(B, gg) : 0.0;  // G_Trapezoid!'s du(u_n)
        for (int b = 0; b < B.nb; ++b) {
            const double* __restrict__ v = B.v[b];
            const double eps = B.eps[b];
            double f[NP], xc = 0.0;
#pragma unroll
            for (int q = 0; q < NP; ++q) {
                double w = 0.0;
                if (s.ok[q]) w = FD ? uu[q] + eps * v[s.off[q]] : v[s.off[q]];  // w = u + eps v, or v
                if (q == 0) xc = w;                                             // the "- u" term
                if constexpr (SCH == 1) {  // G_Midpoint!: α u_n + (1 - α) w; tangent (1 - α) v
                    if (s.ok[q]) w = FD ? B.alpha * gg[q] + (1.0 - B.alpha) * w : (1.0 - B.alpha) * w;
                }
                f[q] = w;
            }
            const double c = f[0];
            if (SCH != 1) xc = c;
            const double lsum = lsum_of<DIM>(B, f);
            double r;
            if constexpr (kind_bratu(KIND)) {
                if constexpr (FD) r = ((lsum + B.lam * nk_exp(c)) - f0) / eps;
                else r = lsum + B.lam * (eu * c);
            } else if constexpr (!FD) {
                r = (SCH == 2 ? B.dt / 2.0 : B.dt) * (B.a * lsum) - xc;
            } else {
                const double g = SCH == 2 ? (unc + (B.dt / 2.0) * (B.a * lsumg + B.a * lsum)) - xc
                                          : (unc + B.dt * (B.a * lsum)) - xc;
                r = (g - f0) / eps;
            }
            B.out[b][o] = r;
        }
    }
}

template <int KIND>
void go_batch(const BArgs& B, int mode, int grid, hipStream_t s) {
    if (mode == MODE_JFD) hipLaunchKernelGGL((k_jv_batch<KIND, MODE_JFD>), dim3(grid), dim3(kBlock), 0, s, B);
    else hipLaunchKernelGGL((k_jv_batch<KIND, MODE_JEXACT>), dim3(grid), dim3(kBlock), 0, s, B);
}

int batch_grid(int64_t n) {
    const int64_t g = (n + kBlock - 1) / kBlock;
    return (int)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

// ------------------------------------------------------------------------------ collect(J)
// distance-2 colouring of the stencil graph: (i + 2j + 3k) mod (2 dim + 1)
__device__ __forceinline__ int color_of(int64_t o, int64_t nx, int64_t ny, int dim) {
    const int64_t i = o % nx, j = (o / nx) % ny, k = o / (nx * ny);
    const int64_t c = dim == 1 ? i : (dim == 2 ? i + 2 * j : i + 2 * j + 3 * k);
    return (int)(c % (2 * dim + 1));
}

__global__ void k_color_probe(BArgs B, int dim) {
    for (int64_t o = (int64_t)blockIdx.x * kBlock + threadIdx.x; o < B.n; o += (int64_t)gridDim.x * kBlock) {
        const int col = color_of(o, B.nx, B.ny, dim);
        for (int b = 0; b < B.nb; ++b) B.out[b][o] = (b == col) ? 1.0 : 0.0;
    }
}

// Column q of J: rows = the stencil points of q (the pattern is symmetric), J[r, q] = probe of
// colour(q) at row r.  Rows sorted ascending (the periodic wrap can put them out of order).
struct ColEntries {
    int64_t row[7];
    double val[7];
    int m;
};
template <int DIM>
__device__ __forceinline__ ColEntries column(const BArgs& B, const double* const* probes, int64_t q) {
    const Nbrs<DIM> s = nbrs<DIM>(B, q);
    const double* pr = probes[color_of(q, B.nx, B.ny, DIM)];
    ColEntries e;
    e.m = 0;
    const int64_t pl = DIM == 1 ? 1 : (DIM == 2 ? B.nx : B.nx * B.ny);
    const int64_t nslow = B.n / pl;
    const int64_t slow = q / pl;
#pragma unroll
    for (int t = 0; t < 2 * DIM + 1; ++t) {
        if (!s.ok[t]) continue;
        int64_t r = s.off[t];
        // the slow-axis neighbour beyond the slab: a ghost plane (no row of this J), or the periodic wrap
        if (t == 2 * DIM - 1 && slow + 1 >= nslow) { if (!B.per) continue; r -= nslow * pl; }
        if (t == 2 * DIM && slow == 0) { if (!B.per) continue; r += nslow * pl; }
        const double v = pr[r];
        if (v != 0.0) {  // collect keeps only the nonzeros (src/Ariadne.jl:155-157)
            int k = e.m++;
            while (k > 0 && e.row[k - 1] > r) { e.row[k] = e.row[k - 1]; e.val[k] = e.val[k - 1]; --k; }
            e.row[k] = r;
            e.val[k] = v;
        }
    }
    return e;
}

struct Probes {
    const double* p[7];
};

// unit vectors e_{j0 + b} (b < nb, j0 + b < n) into the batch's probe vectors
__global__ void k_unit_probe(BArgs B, int64_t j0) {
    for (int64_t o = (int64_t)blockIdx.x * kBlock + threadIdx.x; o < B.n; o += (int64_t)gridDim.x * kBlock)
        for (int b = 0; b < B.nb; ++b) B.out[b][o] = (o == j0 + b) ? 1.0 : 0.0;
}
template <int DIM>
__global__ void k_collect_count(BArgs B, Probes P, int64_t* cnt) {
    for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < B.n; q += (int64_t)gridDim.x * kBlock)
        cnt[q] = column<DIM>(B, P.p, q).m;
}
template <int DIM>
__global__ void k_collect_fill(BArgs B, Probes P, const int64_t* colptr, int64_t* rowval, double* nzval) {
    for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < B.n; q += (int64_t)gridDim.x * kBlock) {
        const ColEntries e = column<DIM>(B, P.p, q);
        const int64_t at = colptr[q];
        for (int t = 0; t < e.m; ++t) {
            rowval[at + t] = e.row[t];
            nzval[at + t] = e.val[t];
        }
    }
}

}  // namespace

// products of J(u) (exact tangent or FD quotient) with nb <= kMaxBatch vectors in one launch;
// ghost planes of u / u_n / every v must be current
int launch_jv_batch(nk_ctx* c, const nk_problem* p, int nb, double* const* out, const double* u,
                    const double* const* v, const double* F0, int mode, const double* eps) {
    if (nb < 1 || nb > kMaxBatch) return fail(c, NK_E_ARG, "launch_jv_batch: 1..8 vectors per launch");
    Geo g;
    NK_TRY(geometry(c, p, &g));
    BArgs B{};
    for (int b = 0; b < nb; ++b) {
        B.out[b] = out[b];
        B.v[b] = v[b];
        B.eps[b] = eps ? eps[b] : 0.0;
    }
    B.u = u; B.F0 = F0; B.un = p->un; B.nb = nb; B.per = p->bc == NK_BC_PERIODIC;
    B.n = g.n; B.nx = p->nx; B.ny = p->ny; B.nz = p->nz;
    B.hx2 = p->hx * p->hx; B.hy2 = p->hy * p->hy; B.hz2 = p->hz * p->hz;
    B.lam = p->lambda; B.a = p->a; B.dt = p->dt; B.alpha = p->alpha;
    const bool heat = nk_is_heat(p->kind), fd = mode == MODE_JFD;
    // algorithmic bytes: per point u / F0 / u_n once, each v read and each product written
    const double words = 2.0 * nb + (fd ? 2.0 + (heat ? 1.0 : 0.0) : (heat ? 0.0 : 1.0));
    const int grid = batch_grid(g.n);
    hipStream_t s = c->stream;
    const int kind = p->kind;
    return launch(c, fd ? "jv_fd_batch" : "jv_exact_batch", 8.0 * words * (double)g.n, [&] {
        switch (kind) {
        case NK_BRATU1D: go_batch<NK_BRATU1D>(B, mode, grid, s); break;
        case NK_BRATU2D: go_batch<NK_BRATU2D>(B, mode, grid, s); break;
        case NK_HEAT2D_EULER: go_batch<NK_HEAT2D_EULER>(B, mode, grid, s); break;
        case NK_HEAT3D_EULER: go_batch<NK_HEAT3D_EULER>(B, mode, grid, s); break;
        case NK_HEAT2D_MIDPOINT: go_batch<NK_HEAT2D_MIDPOINT>(B, mode, grid, s); break;
        case NK_HEAT3D_MIDPOINT: go_batch<NK_HEAT3D_MIDPOINT>(B, mode, grid, s); break;
        case NK_HEAT2D_TRAPEZOID: go_batch<NK_HEAT2D_TRAPEZOID>(B, mode, grid, s); break;
        default: go_batch<NK_HEAT3D_TRAPEZOID>(B, mode, grid, s); break;
        }
    });
}

// collect(J) of a built-in stencil on one rank (exact tangent): CSC arrays, 0-based, on the host.
// Returns NK_E_ARG with *nnz set when cap is too small; 1 when the colouring does not apply (a
// periodic extent not divisible by 2 dim + 1, or < 3): the caller probes unit vectors instead.
int collect_stencil(nk_ctx* c, const nk_problem* p, const double* u, int64_t* colptr, int64_t* rowval, double* nzval,
                    int64_t cap, int64_t* nnz) {
    Geo g;
    NK_TRY(geometry(c, p, &g));
    const int dim = g.dim, ncol = 2 * dim + 1;
    if (p->bc == NK_BC_PERIODIC) {
        const int64_t ext[3] = {p->nx, p->ny, p->nz};
        for (int d = 0; d < dim; ++d)
            if (ext[d] < 3 || ext[d] % ncol != 0) return 1;
    }
    nk_problem geo = *p;
    std::vector<double*> pv(ncol, nullptr), po(ncol, nullptr);
    int rc = NK_OK;
    auto cleanup = [&] {
        for (double* x : pv) if (x) (void)nk_vec_free(c, x);
        for (double* x : po) if (x) (void)nk_vec_free(c, x);
    };
    for (int k = 0; k < ncol && rc == NK_OK; ++k) {
        rc = nk_vec_alloc(c, &geo, &pv[k]);
        if (rc == NK_OK) rc = nk_vec_alloc(c, &geo, &po[k]);
    }
    if (rc != NK_OK) { cleanup(); return rc; }
    BArgs B{};
    B.nb = ncol; B.n = g.n; B.nx = p->nx; B.ny = p->ny; B.nz = p->nz; B.per = p->bc == NK_BC_PERIODIC;
    for (int k = 0; k < ncol; ++k) B.out[k] = pv[k];
    rc = launch(c, "collect_probe", 8.0 * ncol * (double)g.n,
                [&] { hipLaunchKernelGGL(k_color_probe, dim3(batch_grid(g.n)), dim3(kBlock), 0, c->stream, B, dim); });
    for (int k = 0; k < ncol && rc == NK_OK; ++k) rc = halo_exchange(c, p, pv[k]);  // periodic: wrap the ghost planes
    if (rc == NK_OK) rc = halo_exchange(c, p, u);
    if (rc == NK_OK) rc = exchange_un(c, p);
    if (rc == NK_OK) rc = launch_jv_batch(c, p, ncol, po.data(), u, pv.data(), nullptr, MODE_JEXACT, nullptr);
    Probes P{};
    for (int k = 0; k < ncol; ++k) P.p[k] = po[k];
    int64_t* dcnt = nullptr;
    int64_t *drow = nullptr;
    double* dval = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    auto cleanup2 = [&] {
        if (dcnt) (void)hipFree(dcnt);
        if (drow) (void)hipFree(drow);
        if (dval) (void)hipFree(dval);
        if (tmp) (void)hipFree(tmp);
        cleanup();
    };
    if (rc == NK_OK && hipMalloc(&dcnt, sizeof(int64_t) * (size_t)(g.n + 1)) != hipSuccess)
        rc = fail(c, NK_E_NOMEM, "collect: column counts");
    const int grid = batch_grid(g.n);
    if (rc == NK_OK) {
        (void)hipMemsetAsync(dcnt + g.n, 0, sizeof(int64_t), c->stream);
        rc = launch(c, "collect_count", 8.0 * (double)g.n, [&] {
            if (dim == 1) hipLaunchKernelGGL(k_collect_count<1>, dim3(grid), dim3(kBlock), 0, c->stream, B, P, dcnt);
            else if (dim == 2) hipLaunchKernelGGL(k_collect_count<2>, dim3(grid), dim3(kBlock), 0, c->stream, B, P, dcnt);
            else hipLaunchKernelGGL(k_collect_count<3>, dim3(grid), dim3(kBlock), 0, c->stream, B, P, dcnt);
        });
    }
    // exclusive scan of n + 1 counts (the last one 0): colptr[q] = first entry of column q, colptr[n] = nnz
    if (rc == NK_OK && hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, dcnt, dcnt, (int)(g.n + 1), c->stream) != hipSuccess)
        rc = fail(c, NK_E_HIP, "collect: scan size");
    if (rc == NK_OK && hipMalloc(&tmp, tmp_bytes ? tmp_bytes : 1) != hipSuccess) rc = fail(c, NK_E_NOMEM, "collect: scan scratch");
    if (rc == NK_OK && hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, dcnt, dcnt, (int)(g.n + 1), c->stream) != hipSuccess)
        rc = fail(c, NK_E_HIP, "collect: scan");
    int64_t total = 0;
    if (rc == NK_OK && hipMemcpyAsync(&total, dcnt + g.n, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream) != hipSuccess)
        rc = fail(c, NK_E_HIP, "collect: nnz");
    if (rc == NK_OK) rc = nk_sync(c);
    if (rc == NK_OK) {
        *nnz = total;
        if (total > cap) rc = fail(c, NK_E_ARG, "collect: nnz = " + std::to_string(total) + " exceeds cap");
    }
    if (rc == NK_OK && (hipMalloc(&drow, sizeof(int64_t) * (size_t)(total + 1)) != hipSuccess ||
                        hipMalloc(&dval, sizeof(double) * (size_t)(total + 1)) != hipSuccess))
        rc = fail(c, NK_E_NOMEM, "collect: entries");
    if (rc == NK_OK) {
        rc = launch(c, "collect_fill", 24.0 * (double)total, [&] {
            if (dim == 1) hipLaunchKernelGGL(k_collect_fill<1>, dim3(grid), dim3(kBlock), 0, c->stream, B, P, dcnt, drow, dval);
            else if (dim == 2) hipLaunchKernelGGL(k_collect_fill<2>, dim3(grid), dim3(kBlock), 0, c->stream, B, P, dcnt, drow, dval);
            else hipLaunchKernelGGL(k_collect_fill<3>, dim3(grid), dim3(kBlock), 0, c->stream, B, P, dcnt, drow, dval);
        });
    }
    if (rc == NK_OK &&
        (hipMemcpyAsync(colptr, dcnt, sizeof(int64_t) * (size_t)(g.n + 1), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
         hipMemcpyAsync(rowval, drow, sizeof(int64_t) * (size_t)total, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
         hipMemcpyAsync(nzval, dval, sizeof(double) * (size_t)total, hipMemcpyDeviceToHost, c->stream) != hipSuccess))
        rc = fail(c, NK_E_HIP, "collect: copy out");
    if (rc == NK_OK) rc = nk_sync(c);
    cleanup2();
    return rc;
}

// collect(J) by unit-vector probing, as the reference does (src/Ariadne.jl:148-160): user residuals
// (unknown coupling) and periodic grids the colouring does not fit.  O(n^2) host work: n <= 8192.
int collect_unit(nk_ctx* c, const nk_problem* p, const double* u, int transpose, int64_t* colptr, int64_t* rowval,
                 double* nzval, int64_t cap, int64_t* nnz) {
    Geo g;
    NK_TRY(geometry(c, p, &g));
    if (g.n > 8192) return fail(c, NK_E_ARG, "collect(J) by unit probing is limited to n <= 8192 points");
    const bool user = nk_is_user(p->kind);
    nk_problem geo = *p;
    std::vector<double*> pv(kMaxBatch, nullptr), po(kMaxBatch, nullptr);
    int rc = NK_OK;
    for (int k = 0; k < kMaxBatch && rc == NK_OK; ++k) {
        rc = nk_vec_alloc(c, &geo, &pv[k]);
        if (rc == NK_OK) rc = nk_vec_alloc(c, &geo, &po[k]);
    }
    std::vector<double> host((size_t)kMaxBatch * (size_t)g.n);
    int64_t at = 0;
    colptr[0] = 0;
    for (int64_t j0 = 0; j0 < g.n && rc == NK_OK; j0 += kMaxBatch) {
        const int nb = (int)std::min<int64_t>(kMaxBatch, g.n - j0);
        BArgs B{};
        B.nb = nb;
        B.n = g.n;
        for (int b = 0; b < nb; ++b) B.out[b] = pv[b];
        rc = launch(c, "collect_probe", 8.0 * nb * (double)g.n,
                    [&] { hipLaunchKernelGGL(k_unit_probe, dim3(batch_grid(g.n)), dim3(kBlock), 0, c->stream, B, j0); });
        if (rc == NK_OK) {
            if (user || transpose) {
                for (int b = 0; b < nb && rc == NK_OK; ++b)
                    rc = transpose ? nk_jtv(c, p, po[b], u, pv[b]) : nk_jv(c, p, po[b], u, pv[b], nullptr, NK_JV_EXACT, 0.0);
            } else {
                rc = nk_jv_batched(c, p, nb, po.data(), u, pv.data(), nullptr, NK_JV_EXACT, 0.0);
            }
        }
        for (int b = 0; b < nb && rc == NK_OK; ++b) rc = nk_memcpy_d2h(c, host.data() + (size_t)b * g.n, po[b], g.n);
        if (rc == NK_OK) rc = nk_sync(c);
        for (int b = 0; b < nb && rc == NK_OK; ++b) {
            const double* col = host.data() + (size_t)b * g.n;
            for (int64_t i = 0; i < g.n; ++i) {
                if (col[i] != 0.0) {  // src/Ariadne.jl:155-157
                    if (at < cap) {
                        rowval[at] = i;
                        nzval[at] = col[i];
                    }
                    ++at;
                }
            }
            colptr[j0 + b + 1] = at;
        }
    }
    for (double* x : pv) if (x) (void)nk_vec_free(c, x);
    for (double* x : po) if (x) (void)nk_vec_free(c, x);
    if (rc != NK_OK) return rc;
    *nnz = at;
    if (at > cap) return fail(c, NK_E_ARG, "collect: nnz = " + std::to_string(at) + " exceeds cap");
    return NK_OK;
}

}  // namespace nk

using namespace nk;

extern "C" {

int nk_jv_batched(nk_ctx* c, const nk_problem* p, int32_t k, double* const* out, const double* u, const double* const* v,
                  const double* F0, int32_t mode, double eps) {
    if (!c || !p || !out || !u || !v || k < 0) return NK_E_ARG;
    if (mode != NK_JV_EXACT && mode != NK_JV_FD) return fail(c, NK_E_ARG, "bad Jv mode");
    if (k == 0) return NK_OK;
    for (int b = 0; b < k; ++b)
        if (!out[b] || !v[b]) return NK_E_ARG;
    Geo g{};
    if (!nk_is_user(p->kind)) NK_TRY(geometry(c, p, &g));
    // a user residual has no batched kernel, and 3D blocks take their x / y ghost layers from faces the
    // batched kernel does not read: one product per column (each bit-identical to the batched form)
    if (nk_is_user(p->kind) || blocks3d(c, g)) {
        for (int b = 0; b < k; ++b) NK_TRY(nk_jv(c, p, out[b], u, v[b], F0, mode, eps));
        return NK_OK;
    }
    if (mode == NK_JV_FD && !F0) return fail(c, NK_E_ARG, "FD Jv needs F0 = F(u)");
    std::vector<double> e((size_t)k, eps);
    std::vector<char> zero((size_t)k, 0);
    if (mode == NK_JV_FD && eps <= 0.0) {  // per column, as nk_jv chooses it
        double un = 0.0;
        NK_TRY(nk_norm(c, g.n, u, &un));
        for (int b = 0; b < k; ++b) {
            double vn = 0.0;
            NK_TRY(nk_norm(c, g.n, v[b], &vn));
            zero[b] = vn == 0.0;
            e[b] = zero[b] ? 1.0 : std::sqrt(DBL_EPSILON) * std::fmax(1.0, un) / vn;
        }
    }
    NK_TRY(halo_exchange(c, p, u));
    NK_TRY(exchange_un(c, p));
    for (int b = 0; b < k; ++b) NK_TRY(halo_exchange(c, p, v[b]));
    const int md = mode == NK_JV_FD ? MODE_JFD : MODE_JEXACT;
    for (int b0 = 0; b0 < k; b0 += kMaxBatch) {
        const int nb = std::min(kMaxBatch, k - b0);
        NK_TRY(launch_jv_batch(c, p, nb, out + b0, u, v + b0, F0, md, e.data() + b0));
    }
    for (int b = 0; b < k; ++b)
        if (zero[b]) NK_TRY(launch_fill(c, g.n, out[b], 0.0));  // v = 0: nk_jv's result
    return NK_OK;
}

int nk_jtv_batched(nk_ctx* c, const nk_problem* p, int32_t k, double* const* out, const double* u, const double* const* v) {
    if (!c || !p || !out || !u || !v || k < 0) return NK_E_ARG;
    if (!nk_is_user(p->kind))  // symmetric Jacobians: J^T V = J V, the exact tangent
        return nk_jv_batched(c, p, k, out, u, v, nullptr, NK_JV_EXACT, 0.0);
    for (int b = 0; b < k; ++b) NK_TRY(nk_jtv(c, p, out[b], u, v[b]));
    return NK_OK;
}

int nk_jacobian_collect(nk_ctx* c, const nk_problem* p, const double* u, int32_t transpose, int64_t* colptr,
                        int64_t* rowval, double* nzval, int64_t cap, int64_t* nnz) {
    if (!c || !p || !u || !colptr || !nnz || cap < 0 || (cap > 0 && (!rowval || !nzval))) return NK_E_ARG;
    if (c->nranks > 1) return fail(c, NK_E_ARG, "collect(J) of a distributed operator: gather the slabs first");
    if (!nk_is_user(p->kind)) {  // symmetric pattern and values: collect(transpose(J)) == collect(J)
        const int rc = collect_stencil(c, p, u, colptr, rowval, nzval, cap, nnz);
        if (rc != 1) return rc;
    }
    return collect_unit(c, p, u, transpose, colptr, rowval, nzval, cap, nnz);
}

}  // extern "C"
