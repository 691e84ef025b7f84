// nk_stencil.hpp -- what the residual / Jacobian-vector stencils share: the launch arguments (KArgs), the
// per-point arithmetic (point_value, the Laplacian, the FD quotient), the 1D kernel, row loads and cooking,
// x-edges, the XCD-aware tile orders.  The 2D / 3D kernel templates and their dispatch are in
// nk_stencil_kern.hpp; each kind is instantiated in its own translation unit (nk_stencil_inst.hip,
// compiled once per NK_ST_KIND) so the build parallelises; nk_kernels.hip reaches them through the
// stencil_kind_<K> entry points.
#pragma once
#include <cstdio>
#include <type_traits>

#include "nk_device.hpp"

namespace nk {

struct KArgs {
    double* out;
    const double* u;
    const double* v;
    const double* F0;
    const double* un;
    const double* aux;
    double* part;
    int64_t nx, ny, nz;
    double hx2, hy2, hz2, lam, a, dt, eps;
    int tiles_x, tiles_y, rows;
    int fast;            // kbench build only: bit 1 multiplies by reciprocals instead of dividing (not bit-faithful)
    double ihx2, ihy2, ihz2, ieps;
    // fused Arnoldi normalisation: the stencil input is v = src / *vdiv (kdivcopy!, bit-identical),
    // and the block's own points of v are stored to vout (V_k) -- saves the separate divcopy pass
    const double* vdiv;
    double* vout;
    double hd;           // *vdiv, loaded once per block
    double ihd;          // RN(1 / hd), for div_rn
    int fin;             // fold the partials in-kernel (publish)
    double alpha;        // G_Midpoint! α
    int nw;              // 3D: rows (waves) per tile
    int lds3;            // 3D: y-neighbour rows through LDS (k_st3l) instead of per-wave loads (k_st3d)
    int ym;              // 3D: the y-march (k_st3y: NW planes per tile, rows marched, z-neighbours through LDS)
    int lin;             // tiles in dispatch (= address) order instead of XCD-contiguous bands
    int zalt;            // 3D: z-chunks of one tile column dispatched together, odd chunks marching down
    int tile2;           // 2D one-shot LDS tiles of tile2 rows (k_st2t) instead of the row march (0: march)
    double* tpart;       // one-shot tiles with more tiles than kTileParts: per-tile partials (plain stores),
    int group;           //   folded in groups of `group` tiles by k_tile_fold right after the stencil launch
    int f0r;             // 2D FD: F0 = F(u) recomputed from the u rows already loaded (k_st2d<..., F0R>)
    int blk;             // 3D blocks (k_st3l<..., BLK>): x / y ghost layers from the faces at fy / fx
    int nbm;             //   bit s: side s (kHaloSides numbering) has a neighbour
    int64_t fy, fx;      //   offsets of the y-lo / x-lo faces from the interior pointer
    // ghost planes of v through the peers' inboxes inside this launch (halo_tile_exchange): the rank
    // has a lower / upper neighbour whose boundary patch this launch fetches itself
    int hx_lo, hx_hi;
    uint64_t hx_epoch;
    int64_t hx_cap;
    // 3D blocks: all ghost layers of v through the peers' inboxes inside this launch (blk_tile_exchange):
    // the neighbour rank of each side (-1: a physical boundary) and the host-built tile order (exchanging
    // tiles first, partners close together)
    int hx_blk;
    int bnbr[6];
    const int* torder;
};

// What one stencil dispatch launched: the instantiation as rocprofv3 names it (without the anonymous
// namespace and the argument list: the key of profiles/*/pmc_traffic_*.json) and whether it recomputes
// F(u) instead of loading F0 (the byte model and nk_path_info's F0R counts follow it, not the policy)
struct StInst {
    char name[64];
    bool f0r;
};

// per-kind entry points (nk_stencil_inst.hip): launch one stencil kernel of kind K / bind its g_mb
#define NK_ST_DECL(K)                                                                                      \
    StInst stencil_kind_##K(const KArgs& A, int mode, int epi, int vec, int grid, hipStream_t s, bool per); \
    hipError_t stencil_bind_mb_##K(const MbInfo& m);
NK_ST_DECL(1)
NK_ST_DECL(2)
NK_ST_DECL(3)
NK_ST_DECL(4)
NK_ST_DECL(5)
NK_ST_DECL(6)
NK_ST_DECL(7)
NK_ST_DECL(8)
#undef NK_ST_DECL

namespace {

// implicit.jl scheme of a heat kind: 0 G_Euler! (and the Bratu kinds), 1 G_Midpoint!, 2 G_Trapezoid!
template <int KIND>
constexpr int scheme_of() {
    return (KIND == NK_HEAT2D_MIDPOINT || KIND == NK_HEAT3D_MIDPOINT)
               ? 1
               : ((KIND == NK_HEAT2D_TRAPEZOID || KIND == NK_HEAT3D_TRAPEZOID) ? 2 : 0);
}
template <int KIND>
constexpr bool heat_kind() {
    return KIND >= NK_HEAT2D_EULER && KIND <= NK_HEAT3D_TRAPEZOID;
}

// div_rn is used in the Bratu stencil objects only (nk_stencil_inst.hip with NK_ST_KIND 1 / 2: their FD Jv
// 130 -> 126 us, profiles/r04/ab_div_rn.log); elsewhere its guard's compares and exec-mask branches cost
// more than the division sequence they replace (the heat2d FD Jv loop: 304 -> 471 instructions).
#if defined(NK_ST_KIND) && (NK_ST_KIND == NK_BRATU1D || NK_ST_KIND == NK_BRATU2D)
#define NK_ST_DIV_RN 1
#else
#define NK_ST_DIV_RN 0
#endif
// RN(a / b), the IEEE quotient, from yb = RN(1 / b) (computed once: host or kernel prologue): q0 = a yb is
// within an ulp of a / b, the remainder a - b q0 is exact (fma), and one correction q0 + r yb rounds to
// RN(a / b) (Markstein's theorem; round to nearest, no under/overflow -- the operands outside
// 2^-900 <= |a|, |q0| <= 2^1000, zeros included, take the division itself).  3 VALU operations instead of
// the ~10 of a division; bit-identical (also checked on 2.2e8 quotients by tests/test_div_rn.py).
__device__ __forceinline__ double div_rn(double a, double b, double yb) {
#if !NK_ST_DIV_RN
    (void)yb;
    return a / b;
#endif
    const double q0 = a * yb;
    const double r = fma(-q0, b, a);
    const double q1 = fma(r, yb, q0);
    const double aa = fabs(a), aq = fabs(q0);
    if (__builtin_expect(aa >= 0x1p-900 && aq >= 0x1p-900 && aq <= 0x1p1000, 1)) return q1;
    return a / b;
}

__device__ __forceinline__ double vin(const KArgs& A, int64_t o) {
    const double v = A.v[o];
    return A.vdiv ? div_rn(v, A.hd, A.ihd) : v;
}

// ((p - 2c) + m) / h^2 exactly as the reference writes it (div_rn: the same double); the kbench build's
// `fast` variant multiplies by 1/h^2 instead (not bit-faithful)
__device__ __forceinline__ double lapk(const KArgs& A, double c, double p, double m, double h2, double ih2) {
    const double s = (p - 2.0 * c) + m;
#ifdef NK_KBENCH
    if (A.fast & 1) return s * ih2;
    if (A.fast & (1 << 23)) return s / h2;  // A/B: the division instruction sequence
#endif
    return div_rn(s, h2, ih2);
}
// (r - F0) / eps, the FD quotient (kbench `fast`: times 1/eps)
__device__ __forceinline__ double fdq(const KArgs& A, double r, double f0c) {
#ifdef NK_KBENCH
    if (A.fast & 1) return (r - f0c) * A.ieps;
    if (A.fast & (1 << 23)) return (r - f0c) / A.eps;
#endif
    return div_rn(r - f0c, A.eps, A.ieps);
}

template <int MODE>
__device__ __forceinline__ double fieldval(const KArgs& A, int64_t o) {
    if (MODE == MODE_RES) return A.u[o];
    if (MODE == MODE_JEXACT) return vin(A, o);
    return A.u[o] + A.eps * vin(A, o);  // w = u + eps v
}

template <int MODE, int VEC>
__device__ __forceinline__ void fieldvec(const KArgs& A, int64_t o, double* f) {
    if (VEC == 2) {
        if (MODE == MODE_RES) {
            const double2 q = *reinterpret_cast<const double2*>(A.u + o);
            f[0] = q.x; f[1] = q.y;
        } else if (MODE == MODE_JEXACT) {
            const double2 q = *reinterpret_cast<const double2*>(A.v + o);
            f[0] = q.x; f[1] = q.y;
        } else {
            const double2 qu = *reinterpret_cast<const double2*>(A.u + o);
            const double2 qv = *reinterpret_cast<const double2*>(A.v + o);
            f[0] = qu.x + A.eps * qv.x;
            f[1] = qu.y + A.eps * qv.y;
        }
    } else {
        f[0] = fieldval<MODE>(A, o);
    }
}

template <int VEC>
__device__ __forceinline__ void loadvec(const double* __restrict__ p, int64_t o, double* f) {
    if (VEC == 2) {
        const double2 q = *reinterpret_cast<const double2*>(p + o);
        f[0] = q.x; f[1] = q.y;
    } else {
        f[0] = p[o];
    }
}

template <int VEC>
__device__ __forceinline__ void storevec(double* __restrict__ p, int64_t o, const double* f) {
    if (VEC == 2) {
        *reinterpret_cast<double2*>(p + o) = make_double2(f[0], f[1]);
    } else {
        p[o] = f[0];
    }
}

constexpr bool kind_bratu(int k) { return k == NK_BRATU1D || k == NK_BRATU2D; }
// A/B only (-DNK_ST_KEEP_VDIV): keep the runtime v / h test in every instantiation (round 3's form, where
// the instances without the fused normalisation evaluated the division and discarded it)
#ifdef NK_ST_KEEP_VDIV
constexpr bool kKeepVdiv = true;
#else
constexpr bool kKeepVdiv = false;
#endif
// The Bratu k_st2d march evaluates the exp per lane in one pass (XM = 2: the fast phase, and in the rare
// lanes it does not settle the exact phase, divergently, in vector registers); XM = 1 is round 4's first
// form: the fast phase alone, and a wave with an unsettled lane re-running its whole tile with the full
// exp -- about 64 re-runs per 4096^2 launch, and whichever lands in the last round of waves stretches the
// launch by a whole wave lifetime (FD Jv + dot 176 us against 127 us, profiles/r04/ab_lib_single_pass.log).
#ifndef NK_ST2D_BRATU_XM
#define NK_ST2D_BRATU_XM 2
#endif
// Waves per SIMD the Bratu k_st2d kernels are register-allocated for: 4 (<= 128 VGPRs; the cold exact
// phase's registers stay off the hot path).  5 forces spills the march pays for: 147 us against 127 us.
#ifndef NK_ST2D_BRATU_WPE
#define NK_ST2D_BRATU_WPE 4
#endif
#ifndef NK_ST2D_HEAT_CAP  // A/B: occupancy caps for the trapezoid kernels (no gain: profiles/r04/ab_trapezoid_caps.log)
#define NK_ST2D_HEAT_CAP 0
#endif
constexpr int st2d_wpe(int kind, int mode, bool f0r) {
    return kind_bratu(kind) ? NK_ST2D_BRATU_WPE
                            : ((NK_ST2D_HEAT_CAP && kind == NK_HEAT2D_TRAPEZOID)
                                   ? (mode == MODE_RES ? 6 : (f0r ? 4 : 1))
                                   : 1);
}

// The exp table (NKX_T: 128 double-double entries, 2 KB) copied into LDS once per block for the Bratu
// kinds, where every point evaluates exp: read with ds_read, its lookups never wait behind the rows the
// march keeps in flight (a global-memory table would share their in-order vmcnt).  Declares `et`.
#define NK_EXP_LDS(KIND)                                                                              \
    __shared__ double et_lds[kind_bratu(KIND) ? 256 : 2];                                             \
    const double* const et = et_lds;                                                                  \
    if constexpr (kind_bratu(KIND)) {                                                                 \
        for (int i_ = threadIdx.x; i_ < 256; i_ += blockDim.x) et_lds[i_] = (&NKX_T[0][0])[i_];        \
        __syncthreads();                                                                              \
    }

// residual / JVP value at one point from the stencil field (c + neighbours) and centre data.
// lsum = Laplacian-like sum of the stencil field in the reference's association order.  Heat kinds:
// xc = the centre of w = u (+ eps v) -- or of v for the tangent -- before G_Midpoint!'s mixing (the
// "- u" term), unc = u_n, lsumg = the Laplacian sum of u_n (G_Trapezoid!'s du(u_n)).  du = a * lsum:
//   Euler      (u_n + Δt du(w)) - w                      tangent  Δt (a lap(v)) - v
//   Midpoint   (u_n + Δt du(α u_n + (1-α) w)) - w        tangent  Δt (a lap((1-α) v)) - v
//   Trapezoid  (u_n + (Δt/2) (du(u_n) + du(w))) - w      tangent  (Δt/2) (a lap(v)) - v
// et: the exp table (nk_exp.h's NKX_T) in LDS for the Bratu kinds (NK_EXP_LDS), unused otherwise.
// XM = 1: the exp's fast phase only -- a lane it does not settle sets `rare` (its value is then not the
// correctly rounded one, and the caller recomputes: k_st2d's two-pass march); XM = 0: nk_exp_t itself.
template <int KIND, int MODE, int XM = 0>
__device__ __forceinline__ double point_value(const KArgs& A, double c, double lsum, double uc, double unc, double f0c,
                                              double xc, double lsumg, const double* et, bool& rare) {
    if constexpr (KIND == NK_BRATU1D || KIND == NK_BRATU2D) {
#ifdef NK_KBENCH
        if (A.fast & (1 << 20)) {  // kbench A/B only: the platform (ocml) exp, <= 1 ulp off the correctly rounded one
            if (MODE == MODE_JEXACT) return lsum + A.lam * (exp(uc) * c);
            const double r = lsum + A.lam * exp(c);
            return MODE == MODE_JFD ? fdq(A, r, f0c) : r;
        }
#endif
        auto ex = [&](double x) {
#ifdef NK_KBENCH
            if (A.fast & (1 << 22)) {  // kbench diagnosis only: the fast phase's value, no rounding test acted on
                double y;
                (void)nkx_exp_fast(x, et, &y);
                return y;
            }
#endif
// NK_ST_EXP_DIAG (product variant builds for diagnosis only -- wrong answers): 1 the platform exp, 2 no exp,
// the march's floor without the correctly rounded exp (profiles/r05/ab_expdiag.log)
#if defined(NK_ST_EXP_DIAG) && NK_ST_EXP_DIAG == 1
            return exp(x);
#elif defined(NK_ST_EXP_DIAG) && NK_ST_EXP_DIAG == 2  // no exp at all: the march's cost without it
            return x;
#endif
            if constexpr (XM == 1) {
                double y;
                if (!nkx_exp_fast(x, et, &y)) rare = true;
                return y;
            } else if constexpr (XM == 2) {
                return nk_exp_lane(x, et);
            } else {
                return nk_exp_t(x, et);
            }
        };
        if (MODE == MODE_JEXACT) return lsum + A.lam * (ex(uc) * c);  // Enzyme tangent of λ exp(u)
        const double r = lsum + A.lam * ex(c);
        return MODE == MODE_JFD ? fdq(A, r, f0c) : r;
    } else {  // implicit.jl:8-37
        constexpr int SCH = scheme_of<KIND>();
        if (MODE == MODE_JEXACT) return (SCH == 2 ? A.dt / 2.0 : A.dt) * (A.a * lsum) - xc;
        const double r = SCH == 2 ? (unc + (A.dt / 2.0) * (A.a * lsumg + A.a * lsum)) - xc
                                  : (unc + A.dt * (A.a * lsum)) - xc;
        return MODE == MODE_JFD ? fdq(A, r, f0c) : r;
    }
}

template <int EPI>
__device__ __forceinline__ double epilogue(double& val, double ax, double acc) {
    if (EPI == EPI_SUMSQ) return fma(val, val, acc);
    if (EPI == EPI_DOT || EPI == EPI_DOTV || EPI == EPI_DOTVS) return fma(ax, val, acc);
    if (EPI == EPI_RESID) {
        val = ax - val;  // w = b - A x  (kaxpby!(n, 1, b, -1, w))
        return fma(val, val, acc);
    }
    return acc;
}

// ------------------------------------------------------------------------------ 1D stencil
template <int MODE, int EPI>
__global__ __launch_bounds__(kBlock) void k_st1d(KArgs A0) {
    __shared__ double sh[kShN];
    NK_EXP_LDS(NK_BRATU1D)
    KArgs A = A0;
    if constexpr (!kKeepVdiv && EPI != EPI_DOTV && EPI != EPI_DOTVS) A.vdiv = nullptr;  // v / h only with V_k stored
    A.hd = A.vdiv ? *A.vdiv : 1.0;
    A.ihd = 1.0 / A.hd;
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    double acc = 0.0;
    if (i < A.nx) {
        // ghost cells at -1 and nx exist (zero Dirichlet) -- examples/bratu.jl:17-18
        const double c = fieldval<MODE>(A, i), l = fieldval<MODE>(A, i - 1), r = fieldval<MODE>(A, i + 1);
        const double uc = (MODE == MODE_JEXACT) ? A.u[i] : 0.0;
        const double f0 = (MODE == MODE_JFD) ? A.F0[i] : 0.0;
        bool rare_ = false;
        double val = point_value<NK_BRATU1D, MODE>(A, c, lap(c, r, l, A.hx2), uc, 0.0, f0, c, 0.0, et, rare_);
        const double ax = (EPI == EPI_DOT || EPI == EPI_DOTV || EPI == EPI_RESID) ? A.aux[i]
                          : (EPI == EPI_DOTVS ? div_rn(A.v[i], A.hd, A.ihd) : 0.0);
        acc = epilogue<EPI>(val, ax, acc);
        A.out[i] = val;
        if constexpr (MODE != MODE_RES && (EPI == EPI_DOTV || EPI == EPI_DOTVS)) A.vout[i] = div_rn(A.v[i], A.hd, A.ihd);
    }
    if (EPI != EPI_NONE) publish(acc, A.part, A.fin, sh);
}

// ------------------------------------------------------------------------------ row fragments
// VEC consecutive x-points of one row, held by value (no address taken -> stays in VGPRs).
template <int VEC>
struct Row {
    double v[VEC];
};

template <int MODE, int VEC>
__device__ __forceinline__ Row<VEC> field_row(const KArgs& A, int64_t o, bool ok) {
    Row<VEC> r;
    if (ok) {
        if constexpr (VEC % 2 == 0) {
#pragma unroll
            for (int h = 0; h < VEC; h += 2) {
                if constexpr (MODE == MODE_RES) {
                    const double2 q = *reinterpret_cast<const double2*>(A.u + o + h);
                    r.v[h] = q.x; r.v[h + 1] = q.y;
                } else if constexpr (MODE == MODE_JEXACT) {
                    double2 q = *reinterpret_cast<const double2*>(A.v + o + h);
                    if (A.vdiv) { q.x = div_rn(q.x, A.hd, A.ihd); q.y = div_rn(q.y, A.hd, A.ihd); }
                    r.v[h] = q.x; r.v[h + 1] = q.y;
                } else {
                    const double2 qu = *reinterpret_cast<const double2*>(A.u + o + h);
                    double2 qv = *reinterpret_cast<const double2*>(A.v + o + h);
                    if (A.vdiv) { qv.x = div_rn(qv.x, A.hd, A.ihd); qv.y = div_rn(qv.y, A.hd, A.ihd); }
                    r.v[h] = qu.x + A.eps * qv.x;  // w = u + eps v
                    r.v[h + 1] = qu.y + A.eps * qv.y;
                }
            }
        } else {
            r.v[0] = fieldval<MODE>(A, o);
        }
    } else {
#pragma unroll
        for (int k = 0; k < VEC; ++k) r.v[k] = 0.0;
    }
    return r;
}

// NT: non-temporal (streams not re-read before they would be evicted anyway): between two Jv
// launches the MGS passes stream ~16 vectors through the caches.  NK_ST_NT: F(u) loads and V_k
// stores of the fused Jv; NK_ST_NTU: the 2D FD operator's u loads.  Measured A/B on one box: FD Jv
// 141 -> 129.5 -> 127.2 us at 4096^2 (+1.3 % whole bench), heat 8192^2 neutral.  The v (= q) and
// V_1 loads stay cached: q was just written by the last MGS pass, V_1 is re-read by the next one;
// the 3D kernel keeps u cached too (its y-neighbour rows are re-read by the adjacent waves: NT u
// loads cost 12 % at 512^3).
#ifndef NK_ST_NT
#define NK_ST_NT 1
#endif
#ifndef NK_ST_NTU
#define NK_ST_NTU 1
#endif
#ifndef NK_ST_NTN  // u_n (centre-only loads of G_Euler!): +0.2-0.5 % heat 8192^2 / 512^3
#define NK_ST_NTN 1
#endif
typedef double dv2 __attribute__((ext_vector_type(2)));
template <int VEC, bool NT = false>
__device__ __forceinline__ Row<VEC> data_row(const double* __restrict__ p, int64_t o, bool ok) {
    Row<VEC> r;
    if (ok) {
        if constexpr (VEC % 2 == 0) {
#pragma unroll
            for (int h = 0; h < VEC; h += 2) {
                if constexpr (NT) {
                    const dv2 q = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(p + o + h));
                    r.v[h] = q.x; r.v[h + 1] = q.y;
                } else {
                    const double2 q = *reinterpret_cast<const double2*>(p + o + h);
                    r.v[h] = q.x; r.v[h + 1] = q.y;
                }
            }
        } else {
            r.v[0] = p[o];
        }
    } else {
#pragma unroll
        for (int k = 0; k < VEC; ++k) r.v[k] = 0.0;
    }
    return r;
}

template <int VEC, bool NT = false>
__device__ __forceinline__ void store_row(double* __restrict__ p, int64_t o, const Row<VEC>& r) {
    if constexpr (VEC % 2 == 0) {
#pragma unroll
        for (int h = 0; h < VEC; h += 2) {
            if constexpr (NT) __builtin_nontemporal_store(dv2{r.v[h], r.v[h + 1]}, reinterpret_cast<dv2*>(p + o + h));
            else *reinterpret_cast<double2*>(p + o + h) = make_double2(r.v[h], r.v[h + 1]);
        }
    } else {
        p[o] = r.v[0];
    }
}

// ------------------------------------------------------------------------------ 2D stencil
// Raw (un-cooked) loads of one row segment: VEC centre values + one "edge" value per field.  The
// edge load is issued by every lane (no divergence): lane 0 reads column x0-1, lane 63 column
// x0+VEC, the others re-read their own x0 (a cache-hot dummy).  No arithmetic touches the loaded
// registers until the next iteration, so the compiler's s_waitcnt can leave them in flight.
// Periodic kernels (PER) carry a second edge slot: *e = the left edge, *e2 = the right edge (with
// the x-wrap one lane can need both); G = the row of u_n is loaded as well (G_Midpoint! mixes it
// into the stencil field, G_Trapezoid! takes its Laplacian).
template <int MODE, int VEC>
struct RawRow {
    double a[VEC], ae, ae2;  // u (RES, JFD) or v (JEXACT)
    double b[VEC], be, be2;  // v (JFD)
    double g[VEC], ge, ge2;  // u_n (G)
};

// PER (the second edge slot): e2 = false skips its loads (wave-uniform: no VMEM instruction issued) -- a 3D
// block's x-hi face travels in the first slot except in a one-lane last tile
template <int MODE, int VEC, bool EDGE = true, bool G = false, bool PER = false, bool NTU = false>
__device__ __forceinline__ RawRow<MODE, VEC> load_raw(const KArgs& A, int64_t o, int64_t oe, int64_t oe2 = 0, bool e2 = true) {
    RawRow<MODE, VEC> r;
    const double* __restrict__ pa = (MODE == MODE_JEXACT) ? A.v : A.u;
    if constexpr (VEC % 2 == 0) {
#pragma unroll
        for (int h = 0; h < VEC; h += 2) {
            if constexpr (NTU && MODE == MODE_JFD) {
                const dv2 q = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(pa + o + h));
                r.a[h] = q.x; r.a[h + 1] = q.y;
            } else {
                const double2 q = *reinterpret_cast<const double2*>(pa + o + h);
                r.a[h] = q.x; r.a[h + 1] = q.y;
            }
        }
    } else {
        r.a[0] = pa[o];
    }
    if constexpr (EDGE) r.ae = pa[oe];
    else r.ae = 0.0;
    if constexpr (EDGE && PER) r.ae2 = e2 ? pa[oe2] : 0.0;
    if constexpr (MODE == MODE_JFD) {
        if constexpr (VEC % 2 == 0) {
#pragma unroll
            for (int h = 0; h < VEC; h += 2) {
                const double2 q = *reinterpret_cast<const double2*>(A.v + o + h);
                r.b[h] = q.x; r.b[h + 1] = q.y;
            }
        } else {
            r.b[0] = A.v[o];
        }
        if constexpr (EDGE) r.be = A.v[oe];
        else r.be = 0.0;
        if constexpr (EDGE && PER) r.be2 = e2 ? A.v[oe2] : 0.0;
    }
    if constexpr (G) {
        if constexpr (VEC % 2 == 0) {
#pragma unroll
            for (int h = 0; h < VEC; h += 2) {
                const double2 q = *reinterpret_cast<const double2*>(A.un + o + h);
                r.g[h] = q.x; r.g[h + 1] = q.y;
            }
        } else {
            r.g[0] = A.un[o];
        }
        if constexpr (EDGE) r.ge = A.un[oe];
        else r.ge = 0.0;
        if constexpr (EDGE && PER) r.ge2 = e2 ? A.un[oe2] : 0.0;
    }
    return r;
}

// the same for a ghost row / plane whose v values are in my inbox (ib, indexed by the in-plane
// position p) while u and u_n stay in memory (o); only centres are read -- a ghost row / plane is
// only ever a y / z neighbour, its x-edges are never used
template <int MODE, int VEC, bool G = false>
__device__ __forceinline__ RawRow<MODE, VEC> load_raw_ib(const KArgs& A, const uint64_t* ib, int64_t o, int64_t p) {
    RawRow<MODE, VEC> r;
#pragma unroll
    for (int h = 0; h < VEC; ++h) {
        if constexpr (MODE == MODE_JEXACT) r.a[h] = ld_inbox(ib + p + h);
        else r.a[h] = A.u[o + h];
        if constexpr (MODE == MODE_JFD) r.b[h] = ld_inbox(ib + p + h);
        if constexpr (G) r.g[h] = A.un[o + h];
    }
    r.ae = r.ae2 = 0.0;
    r.be = r.be2 = 0.0;
    r.ge = r.ge2 = 0.0;
    return r;
}

// the u part of a raw FD row (u centres, edges, u_n) as a residual row: cooked as MODE_RES it is the
// stencil field the residual kernel evaluates F(u) on (the F0R kernels recompute F0 from it)
template <int MODE, int VEC>
__device__ __forceinline__ RawRow<MODE_RES, VEC> as_res_row(const RawRow<MODE, VEC>& r) {
    RawRow<MODE_RES, VEC> q;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        q.a[k] = r.a[k];
        q.g[k] = r.g[k];
    }
    q.ae = r.ae;
    q.ae2 = r.ae2;
    q.ge = r.ge;
    q.ge2 = r.ge2;
    return q;
}

// cooked stencil field of a row: centres, the lane's edge value(s), and (fused normalisation) v / h
template <int VEC>
struct Field {
    double c[VEC], e, e2;    // the stencil field (G_Midpoint!: α u_n + (1-α) w); edges (e2: PER right edge)
    double vn[VEC];          // v / h (the stored basis vector)
    double x[VEC];           // w = u (+ eps v) or v before the midpoint mixing: the "- u" term
    double g[VEC], ge, ge2;  // u_n (G)
};

struct WV {
    double w, v;  // the stencil input w = u (+ eps v) or v, and v / h
};
template <int MODE>
__device__ __forceinline__ WV cook_w(const KArgs& A, double ra, double rb, bool div) {
    WV r;
    if constexpr (MODE == MODE_RES) {
        r.v = 0.0;
        r.w = ra;
    } else if constexpr (MODE == MODE_JEXACT) {
        r.v = div ? div_rn(ra, A.hd, A.ihd) : ra;
        r.w = r.v;
    } else {
        r.v = div ? div_rn(rb, A.hd, A.ihd) : rb;
        r.w = ra + A.eps * r.v;  // w = u + eps v
    }
    return r;
}

template <int MODE, int SCH>
__device__ __forceinline__ double mix(const KArgs& A, double w, double g) {
    if constexpr (SCH != 1) return w;
    // G_Midpoint!: uuₙ .= α .* uₙ .+ (1 - α) .* u; its tangent (u_n has a zero shadow) is (1 - α) v
    else if constexpr (MODE == MODE_JEXACT) return (1.0 - A.alpha) * w;
    else return A.alpha * g + (1.0 - A.alpha) * w;
}

template <int MODE, int VEC, int SCH = 0, bool G = false, bool PER = false>
__device__ __forceinline__ Field<VEC> cook(const KArgs& A, const RawRow<MODE, VEC>& r, bool act, bool edge_ok,
                                           bool edge_ok2 = false) {
    Field<VEC> f;
    const bool div = A.vdiv != nullptr;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        const WV q = cook_w<MODE>(A, r.a[k], MODE == MODE_JFD ? r.b[k] : 0.0, div);
        const double w = q.w;
        f.vn[k] = q.v;
        f.x[k] = w;
        f.c[k] = mix<MODE, SCH>(A, w, G ? r.g[k] : 0.0);
        if constexpr (G) f.g[k] = r.g[k];
        if (!act) {  // lanes past the row end act as the zero boundary for their neighbour
            f.c[k] = 0.0;
            if constexpr (G) f.g[k] = 0.0;
        }
    }
    const double e = mix<MODE, SCH>(A, cook_w<MODE>(A, r.ae, MODE == MODE_JFD ? r.be : 0.0, div).w, G ? r.ge : 0.0);
    f.e = edge_ok ? e : 0.0;
    if constexpr (G) f.ge = edge_ok ? r.ge : 0.0;
    if constexpr (PER) {
        const double e2 = mix<MODE, SCH>(A, cook_w<MODE>(A, r.ae2, MODE == MODE_JFD ? r.be2 : 0.0, div).w, G ? r.ge2 : 0.0);
        f.e2 = edge_ok2 ? e2 : 0.0;
        if constexpr (G) f.ge2 = edge_ok2 ? r.ge2 : 0.0;
    }
    return f;
}

// x-edge geometry of one lane.  Without PER: lane 0 reads column x0-1, lane 63 column x0+VEC (zero
// beyond the grid).  With PER (bc_periodic!): lane 0 reads its left neighbour into e (column nx-1 at
// x0 = 0), and lane 63 -- or the lane holding the last column -- its right neighbour into e2
// (column 0 after the last column).
struct XEdge {
    int64_t de, de2;
    bool ok, ok2, rwrap;
};
template <int VEC, bool PER>
__device__ __forceinline__ XEdge x_edge(int lane, bool act, int64_t x0, int64_t nx) {
    XEdge x{};
    if constexpr (!PER) {
        const bool left_ok = lane == 0 && act && x0 >= 1;
        const bool right_ok = lane == 63 && act && x0 + VEC < nx;
        x.de = left_ok ? -1 : (right_ok ? VEC : 0);  // edge element offset (0: dummy)
        x.ok = left_ok || right_ok;
        x.de2 = 0;
        x.ok2 = false;
        x.rwrap = false;
    } else {
        x.ok = lane == 0 && act;
        x.de = x.ok ? (x0 >= 1 ? -1 : nx - 1) : 0;
        x.rwrap = act && x0 + VEC == nx;
        x.ok2 = act && ((lane == 63 && x0 + VEC < nx) || x.rwrap);
        x.de2 = x.ok2 ? (x.rwrap ? -x0 : VEC) : 0;
    }
    return x;
}

// Block -> tile.  Tiles go to the 8 XCDs in contiguous bands (b % 8 is the XCD a block lands on), so
// vertically adjacent tiles share an L2.  With ghost planes exchanged inside the launch (hx_lo / hx_hi)
// the tiles at the slab's ends come first -- the lower band, then the upper band: they push this rank's
// boundary patch at once and wait for the neighbour's, which the neighbour's launch also issues first.
// Dispatched last (in address order), a lower tile would wait on a neighbour whose upper tiles start
// only when most of ITS launch is done -- a chain along the ranks whenever a launch has more tiles than
// the GPU holds at once.  `band` = tiles per plane / row band, `nband` = bands.
// XCD band of dispatch index i of n: block i lands on XCD i % 8 and takes the (i / 8)-th tile of that
// XCD's contiguous band (the last n % 8 blocks in dispatch order)
__device__ __forceinline__ int xcd_band(int i, int n) {
    const int n8 = n & ~7;
    return i < n8 ? (i & 7) * (n8 >> 3) + (i >> 3) : i;
}
__device__ __forceinline__ int tile_of(int b, int nb, int band, int nband, int lo, int hi, int lin) {
    auto xcd = [lin](int i, int n) { return lin ? i : xcd_band(i, n); };
    const int nl = lo ? band : 0, nh = (hi && nband > 1) ? band : 0;
    if (nl + nh == 0) return xcd(b, nb);
    if (b < nl) return b;
    if (b < nl + nh) return (nband - 1) * band + (b - nl);
    return xcd(b - nl - nh, nb - nl - nh) + nl;
}
// 3D block -> (z-chunk tz, tile txy of the plane).  zcol: an XCD's band holds whole tile columns -- all
// z-chunks of one column at consecutive band positions, the columns in y order -- so the chunks of a
// column run at the same time on one L2.  With odd chunks marching downwards (k_st3l, A.zalt) every
// chunk boundary is then read by both of its chunks at the same step (both at their start or both at
// their end), and the z-halo planes come from L2 instead of a second trip to memory; y-adjacent
// columns sit next to each other in the band, so the y-halo rows stay shared as well.  The slab-end
// chunks of the in-launch ghost-plane exchange still come first (tile_of).
__device__ __forceinline__ void tile3_of(int b, int nb, int tiles_x, int tiles_y, int nzc, int lo, int hi, int zcol,
                                         int& tz, int& txy) {
    const int tpl = tiles_x * tiles_y;
    if (zcol == 0 || zcol == 2) {  // plane-major (2: with the odd chunks marching down)
        const int t = tile_of(b, nb, tpl, nzc, lo, hi, 0);
        tz = t / tpl;
        txy = t % tpl;
        return;
    }
    const int nl = lo ? tpl : 0, nh = (hi && nzc > 1) ? tpl : 0;
    if (b < nl) {
        tz = 0;
        txy = b;
        return;
    }
    if (b < nl + nh) {
        tz = nzc - 1;
        txy = b - nl;
        return;
    }
    const int zl = nl ? 1 : 0, nzi = nzc - zl - (nh ? 1 : 0);  // > 0 here
    const int L = xcd_band(b - nl - nh, nb - nl - nh);
    if (zcol == 3) {  // pairs of chunks (2m, 2m + 1) of one tile at consecutive band positions, plane-major otherwise
        const int full = nzi / 2 * 2 * tpl;  // band positions of the full pairs
        if (L >= full) {  // an odd chunk count: the last chunk has no partner
            tz = zl + nzi - 1;
            txy = L - full;
            return;
        }
        const int pr = L >> 1;
        tz = zl + 2 * (pr / tpl) + (L & 1);
        txy = pr % tpl;
        return;
    }
    tz = zl + L % nzi;
    const int col = L / nzi;
    txy = (col % tiles_y) * tiles_x + col / tiles_y;
}

// one-lane shifts across the whole wave as DPP moves (gfx9's wave_shr:1 / wave_shl:1): a VALU op per
// 32-bit half, where __shfl_up / __shfl_down go through the LDS crossbar (ds_bpermute) and an lgkmcnt
// wait.  The lane with no source (0 resp. 63) keeps 0; x_nbrs overrides it with its edge value.
// Opt-in (-DNK_XNBR_DPP=1): bitwise and neutral on every workload measured (profiles/r04/README.md).
#ifndef NK_XNBR_DPP
#define NK_XNBR_DPP 0
#endif
__device__ __forceinline__ double wave_shr1(double x) {  // lane i <- lane i - 1
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x138, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_shl1(double x) {  // lane i <- lane i + 1
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x130, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x130, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

// west / east neighbours of the VEC points of a lane: lane shifts, the wave-edge lanes' edge values
struct LR {
    double l, r;
};
// BLK (3D blocks): lane 0's first slot is its left neighbour (in-array or the x-lo face), lane 63's and
// the x-hi face lane's (rwrap) the right one; only a one-lane last tile (lane 0 on both) uses the second
template <bool PER, bool BLK = false>
__device__ __forceinline__ LR x_nbrs(const KArgs& A, double cfirst, double clast, double e, double e2, int lane,
                                     bool rwrap) {
    LR o;
    (void)A;
#if NK_XNBR_DPP
    o.l = wave_shr1(clast);
    o.r = wave_shl1(cfirst);
#else
    o.l = __shfl_up(clast, 1, 64);
    o.r = __shfl_down(cfirst, 1, 64);
#endif
    if (lane == 0) o.l = e;
    if constexpr (BLK) {
        if (rwrap) o.r = lane == 0 ? e2 : e;
        else if (lane == 63) o.r = e;
    } else if constexpr (PER) {
        if (lane == 63 || rwrap) o.r = e2;
    } else {
        if (lane == 63) o.r = e;
    }
    return o;
}

}  // namespace
}  // namespace nk
