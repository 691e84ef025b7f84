// nk_stencil.hpp -- the residual / Jacobian-vector stencil kernels (1D, 2D, 3D; every problem kind,
// mode and fused epilogue) and their compile-time dispatch.  Each kind is instantiated in its own
// translation unit (nk_stencil_inst.hip, compiled once per NK_ST_KIND) so the build parallelises;
// nk_kernels.hip reaches them through stencil_kind_launch().
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

// Block = 256 threads x VEC columns (one row segment), marching A.rows rows in y.  Pipeline: at
// iteration j the raw loads of row j+2 and the centre operands of row j+1 are issued, row j+1's
// raw data (issued one iteration earlier) is cooked, and row j is computed from registers.
// F0R (FD only): F0 = F(u) is recomputed here -- the u rows are loaded for w = u + eps v anyway -- with
// exactly the residual kernel's arithmetic (the u field cooked as MODE_RES, the same Laplacian and
// point_value), so (F(w) - F(u)) / eps is bit-identical to loading the F0 that kernel stored, and
// 8 B/pt less is read.  Valid only when F0 IS that residual of this u (the Newton loop's res).
template <int KIND, int MODE, int EPI, int VEC, bool PER = false, bool F0R = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(st2d_wpe(KIND, MODE, F0R))))
void k_st2d(KArgs A0) {
    __shared__ double sh[kShN];
    NK_EXP_LDS(KIND)
    KArgs A = A0;
    if constexpr (!kKeepVdiv && EPI != EPI_DOTV && EPI != EPI_DOTVS) A.vdiv = nullptr;  // v / h only with V_k stored
    A.hd = A.vdiv ? *A.vdiv : 1.0;
    A.ihd = 1.0 / A.hd;
    constexpr int SCH = scheme_of<KIND>();
    constexpr bool kG = SCH != 0 && MODE != MODE_JEXACT;  // u_n rows with the stencil field
    const int lane = threadIdx.x & 63;
    const int nb = gridDim.x, b = blockIdx.x;
    const int t = tile_of(b, nb, A.tiles_x, A.tiles_y, A.hx_lo, A.hx_hi, A.lin);  // (lin: address order)
    const int tx = t % A.tiles_x, ty = t / A.tiles_x;
    const int64_t nx = A.nx, ny = A.ny;
    const int64_t x0 = (int64_t)tx * (kBlock * VEC) + (int64_t)threadIdx.x * VEC;
    const bool act = x0 < nx;
    const int64_t xc = act ? x0 : 0;  // clamped column: every load stays inside the allocation
    const XEdge xe = x_edge<VEC, PER>(lane, act, x0, nx);
    const int64_t de = xe.de, de2 = xe.de2;
    const bool edge_ok = xe.ok, edge_ok2 = xe.ok2;
    const int64_t y0 = (int64_t)ty * A.rows;
    const int64_t y1 = y0 + A.rows < ny ? y0 + A.rows : ny;
    // ghost rows of v from the neighbours' patches, fetched by this launch (tiles at the slab's ends)
    const uint64_t* ib_lo = nullptr;
    const uint64_t* ib_hi = nullptr;
    if constexpr (MODE != MODE_RES && !PER) {
        const HaloTile ht{A.hx_lo && y0 == 0 && y0 < ny, A.hx_hi && y1 == ny && y0 < ny};
        if (ht.lo || ht.hi) {  // block-uniform
            const int64_t ca = (int64_t)tx * (kBlock * VEC), cb = ca + kBlock * VEC < nx ? ca + kBlock * VEC : nx;
            if (halo_tile_exchange(A.v, nx, ny, nx, 0, 1, ca, cb, tx, ht, A.hx_epoch, A.hx_cap, kBlock)) {
                const int par = (int)(A.hx_epoch & 1);
                if (ht.lo) ib_lo = halo_inbox(g_mb.self, par, 0, A.hx_cap);
                if (ht.hi) ib_hi = halo_inbox(g_mb.self, par, 1, A.hx_cap);
            }
        }
    }
    constexpr bool kU = MODE == MODE_JEXACT && KIND == NK_BRATU2D;
    constexpr bool kUn = KIND == NK_HEAT2D_EULER && MODE != MODE_JEXACT;
    constexpr bool kF0 = MODE == MODE_JFD && !F0R;
    constexpr bool kR = MODE == MODE_JFD && F0R;  // the u field, cooked as the residual kernel cooks it
    constexpr bool kAx = EPI == EPI_DOT || EPI == EPI_DOTV || EPI == EPI_RESID;
    auto as_res = [](const RawRow<MODE, VEC>& r) { return as_res_row<MODE, VEC>(r); };
    constexpr bool vout = MODE != MODE_RES && (EPI == EPI_DOTV || EPI == EPI_DOTVS);  // fused kdivcopy!: V_k stored
    double acc = 0.0;
    // The march as a lambda over XM: the Bratu kinds run it first with the exp's fast phase alone (XM = 1,
    // no exact phase in the loop: its scalar registers would otherwise spill the loop's invariants); a
    // wave any of whose lanes the rounding test did not settle (about one wave-tile in 60) runs its tile
    // again with the full exp (XM = 0), overwriting the same outputs and its partial sum -- so every
    // stored value and partial is the one a single exact pass computes.
    auto march = [&](auto xm_) -> bool {
    constexpr int XM = decltype(xm_)::value;
    bool rare = false;
    if (y0 < ny) {
        // rows y0-1 (ghost plane when y0 = 0) and y0 cooked up front; row y0+1 raw in flight
        const RawRow<MODE, VEC> rm0 =
            ib_lo ? load_raw_ib<MODE, VEC, kG>(A, ib_lo, (y0 - 1) * nx + xc, xc)
                  : load_raw<MODE, VEC, true, kG, PER, NK_ST_NTU>(A, (y0 - 1) * nx + xc, (y0 - 1) * nx + xc + de, (y0 - 1) * nx + xc + de2);
        const RawRow<MODE, VEC> rc0 =
            load_raw<MODE, VEC, true, kG, PER, NK_ST_NTU>(A, y0 * nx + xc, y0 * nx + xc + de, y0 * nx + xc + de2);
        Field<VEC> fm = cook<MODE, VEC, SCH, kG, PER>(A, rm0, act, false, false);
        Field<VEC> fc = cook<MODE, VEC, SCH, kG, PER>(A, rc0, act, edge_ok, edge_ok2);
        Field<VEC> um{}, uc_{};  // F0R: the u field of rows j-1, j
        if constexpr (kR) {
            um = cook<MODE_RES, VEC, SCH, kG, PER>(A, as_res(rm0), act, false, false);
            uc_ = cook<MODE_RES, VEC, SCH, kG, PER>(A, as_res(rc0), act, edge_ok, edge_ok2);
        }
        RawRow<MODE, VEC> rp =
            (ib_hi && y0 + 1 == ny) ? load_raw_ib<MODE, VEC, kG>(A, ib_hi, (y0 + 1) * nx + xc, xc)
                                    : load_raw<MODE, VEC, true, kG, PER, NK_ST_NTU>(A, (y0 + 1) * nx + xc, (y0 + 1) * nx + xc + de, (y0 + 1) * nx + xc + de2);
        Row<VEC> uc{}, unc{}, f0c{}, ax{};
        {
            const int64_t o = y0 * nx + xc;
            if constexpr (kU) uc = data_row<VEC>(A.u, o, true);
            if constexpr (kUn) unc = data_row<VEC, NK_ST_NTN>(A.un, o, true);
            if constexpr (kF0) f0c = data_row<VEC, NK_ST_NT>(A.F0, o, true);
            if constexpr (kAx) ax = data_row<VEC>(A.aux, o, true);
        }
        for (int64_t j = y0; j < y1; ++j) {
            const int64_t o = j * nx + xc;
            // ---- issue: raw row j+2 (rows up to ny are the ghost plane; y1 <= ny keeps j+2 <= ny+1
            //      in range only when j+1 < y1, so clamp to row j+1 otherwise)
            const int64_t r2 = (j + 1 < y1) ? j + 2 : j + 1;  // (ny: the upper ghost row)
            const int64_t o2 = r2 * nx + xc;
            const RawRow<MODE, VEC> rpp = (ib_hi && r2 == ny) ? load_raw_ib<MODE, VEC, kG>(A, ib_hi, o2, xc)
                                                              : load_raw<MODE, VEC, true, kG, PER, NK_ST_NTU>(A, o2, o2 + de, o2 + de2);
            Row<VEC> ucn{}, uncn{}, f0cn{}, axn{};
            const int64_t o1 = (j + 1 < y1) ? o + nx : o;
            if constexpr (kU) ucn = data_row<VEC>(A.u, o1, true);
            if constexpr (kUn) uncn = data_row<VEC, NK_ST_NTN>(A.un, o1, true);
            if constexpr (kF0) f0cn = data_row<VEC, NK_ST_NT>(A.F0, o1, true);
            if constexpr (kAx) axn = data_row<VEC>(A.aux, o1, true);
            // ---- cook row j+1 (its loads were issued one iteration ago)
            const Field<VEC> fp = cook<MODE, VEC, SCH, kG, PER>(A, rp, act, edge_ok && j + 1 < ny, edge_ok2 && j + 1 < ny);
            Field<VEC> up{};
            LR un_{};
            if constexpr (kR) {
                up = cook<MODE_RES, VEC, SCH, kG, PER>(A, as_res(rp), act, edge_ok && j + 1 < ny, edge_ok2 && j + 1 < ny);
                un_ = x_nbrs<PER>(A, uc_.c[0], uc_.c[VEC - 1], uc_.e, uc_.e2, lane, xe.rwrap);
            }
            // ---- compute row j from registers
            const LR xn = x_nbrs<PER>(A, fc.c[0], fc.c[VEC - 1], fc.e, fc.e2, lane, xe.rwrap);
            const double lft = xn.l, rgt = xn.r;
            double glft = 0.0, grgt = 0.0;
            if constexpr (SCH == 2 && kG) {
                const LR gn = x_nbrs<PER>(A, fc.g[0], fc.g[VEC - 1], fc.ge, fc.ge2, lane, xe.rwrap);
                glft = gn.l;
                grgt = gn.r;
            }
            if (act) {
                Row<VEC> val;
#pragma unroll
                for (int k = 0; k < VEC; ++k) {
                    const double w = (k == 0) ? lft : fc.c[k == 0 ? 0 : k - 1];
                    const double e = (k == VEC - 1) ? rgt : fc.c[k == VEC - 1 ? k : k + 1];
                    const double c = fc.c[k];
                    const double lsum = lapk(A, c, e, w, A.hx2, A.ihx2) + lapk(A, c, fp.c[k], fm.c[k], A.hy2, A.ihy2);
                    double lsumg = 0.0;
                    if constexpr (SCH == 2 && kG) {
                        const double gw = (k == 0) ? glft : fc.g[k == 0 ? 0 : k - 1];
                        const double ge = (k == VEC - 1) ? grgt : fc.g[k == VEC - 1 ? k : k + 1];
                        lsumg = lapk(A, fc.g[k], ge, gw, A.hx2, A.ihx2) + lapk(A, fc.g[k], fp.g[k], fm.g[k], A.hy2, A.ihy2);
                    }
                    const double unk = kG ? fc.g[k] : unc.v[k];
                    double f0 = f0c.v[k];
                    if constexpr (kR) {  // F(u) at this point, as the residual kernel evaluates it
                        const double uw = (k == 0) ? un_.l : uc_.c[k == 0 ? 0 : k - 1];
                        const double ue = (k == VEC - 1) ? un_.r : uc_.c[k == VEC - 1 ? k : k + 1];
                        const double ucc = uc_.c[k];
                        const double lsu = lapk(A, ucc, ue, uw, A.hx2, A.ihx2) + lapk(A, ucc, up.c[k], um.c[k], A.hy2, A.ihy2);
                        f0 = point_value<KIND, MODE_RES, XM>(A, ucc, lsu, 0.0, unk, 0.0, SCH == 1 ? uc_.x[k] : ucc, lsumg, et, rare);
                    }
                    double r = point_value<KIND, MODE, XM>(A, c, lsum, uc.v[k], unk, f0, SCH == 1 ? fc.x[k] : c, lsumg, et, rare);
                    acc = epilogue<EPI>(r, EPI == EPI_DOTVS ? fc.vn[k] : ax.v[k], acc);
                    val.v[k] = r;
                }
                store_row<VEC>(A.out, o, val);
                if (vout) {
                    Row<VEC> vn;
#pragma unroll
                    for (int k = 0; k < VEC; ++k) vn.v[k] = fc.vn[k];
                    store_row<VEC, NK_ST_NT>(A.vout, o, vn);
                }
            }
            fm = fc;
            fc = fp;
            if constexpr (kR) {
                um = uc_;
                uc_ = up;
            }
            rp = rpp;
            uc = ucn;
            unc = uncn;
            f0c = f0cn;
            ax = axn;
        }
    }
    return rare;
    };
    if constexpr (kind_bratu(KIND)) {
#if NK_ST2D_BRATU_XM == 2
        (void)march(std::integral_constant<int, 2>{});
#else
        if (__ballot(march(std::integral_constant<int, 1>{}))) {  // wave-uniform
            acc = 0.0;
            (void)march(std::integral_constant<int, 0>{});
        }
#endif
    } else {
        (void)march(std::integral_constant<int, 0>{});
    }
    if constexpr (EPI != EPI_NONE) publish(acc, A.part, A.fin, sh, t);
}

// 3D blocks: the ghost layers of v through the peers' inboxes INSIDE the Jv launch (KArgs::hx_blk) instead of a
// separate k_faces_ipc launch before it.  Tile (tx, ty, tz) owns one patch of every block face it touches: its
// rows x columns of the first / last plane (z), its planes x columns of the first / last row (y), its planes x
// rows of the first / last column (x).  It pushes each patch into that neighbour's inbox at the face layout
// k_faces_ipc uses (system-scope stores, drained), raises the patch's flag there, waits for the neighbour's
// flag of the same patch in its own region, and copies the neighbour's patch into v's ghost plane / face --
// where the march then reads it exactly as after k_faces_ipc, so the arithmetic and the tile-indexed
// partials do not change.  Neighbours share the face's extents and the tiling along it (z-chunks of a fixed
// size, 4-row tiles, 64 VEC columns), so the patch numbers pair up.  Only this tile reads the layers it
// copies (the x-face slots of its rows / planes, the halo rows of its planes, the ghost plane under its
// rows and columns).  The host dispatches the exchanging tiles first, partners within one grid's residency.
template <int NW, int VEC>
__device__ bool blk_tile_exchange(const KArgs& A, int tx, int ty, int tz, int64_t z0, int64_t z1, int nzc) {
    __shared__ int bx_ok;
    const int64_t nx = A.nx, ny = A.ny, nz = A.nz, pl = nx * ny;
    const int64_t ra = (int64_t)ty * NW, rb = ra + NW < ny ? ra + NW : ny;
    const int64_t ca = (int64_t)tx * (64 * VEC), cb = ca + 64 * VEC < nx ? ca + 64 * VEC : nx;
    const int par = (int)(A.hx_epoch & 1);
    constexpr int nthr = 64 * NW;
    // (constant indices only: a dynamic index into the KArgs copy would put it in scratch)
    auto nbr = [&](int s) -> int {
        switch (s) {
        case 0: return A.bnbr[0];
        case 1: return A.bnbr[1];
        case 2: return A.bnbr[2];
        case 3: return A.bnbr[3];
        case 4: return A.bnbr[4];
        default: return A.bnbr[5];
        }
    };
    auto touches = [&](int s) -> bool {
        if (nbr(s) < 0) return false;
        switch (s) {
        case 0: return tz == 0;
        case 1: return tz == nzc - 1;
        case 2: return ty == 0;
        case 3: return ty == A.tiles_y - 1;
        case 4: return tx == 0;
        default: return tx == A.tiles_x - 1;
        }
    };
    auto plen = [&](int s) -> int64_t { return s < 2 ? (rb - ra) * (cb - ca) : (s < 4 ? (z1 - z0) * (cb - ca) : (z1 - z0) * (rb - ra)); };
    // element q of side s's patch: its index f in the face layout (z: j nx + i, y: k nx + i, x: k ny + j) and
    // the offset of my own boundary value in v
    auto at = [&](int s, int64_t q, int64_t& f, int64_t& src) {
        if (s < 2) {
            const int64_t w = cb - ca, j = ra + q / w, i = ca + q % w;
            f = j * nx + i;
            src = (s == 0 ? 0 : (nz - 1) * pl) + f;
        } else if (s < 4) {
            const int64_t w = cb - ca, k = z0 + q / w, i = ca + q % w;
            f = k * nx + i;
            src = k * pl + (s == 2 ? 0 : ny - 1) * nx + i;
        } else {
            const int64_t w = rb - ra, k = z0 + q / w, j = ra + q % w;
            f = k * ny + j;
            src = k * pl + j * nx + (s == 4 ? 0 : nx - 1);
        }
    };
    auto flag_of = [&](int s) -> int { return s < 2 ? ty * A.tiles_x + tx : (s < 4 ? tz * A.tiles_x + tx : tz * A.tiles_y + ty); };
    double* v = const_cast<double*>(A.v);
#pragma unroll
    for (int s = 0; s < kHaloSides; ++s) {  // block-uniform
        if (!touches(s)) continue;
        uint64_t* dst = halo_inbox(g_mb.peers[nbr(s)], par, s ^ 1, A.hx_cap);
        const int64_t len = plen(s);
        for (int64_t q = threadIdx.x; q < len; q += nthr) {
            int64_t f, src;
            at(s, q, f, src);
            __hip_atomic_store(dst + f, (uint64_t)__double_as_longlong(v[src]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every thread drains its stores before the flags
    __syncthreads();
    if (threadIdx.x < 64) {  // lane s raises side s's flag and polls its own: the sides' round trips in parallel
        const int s = (int)threadIdx.x;
        const bool mine = s < kHaloSides && touches(s);
        if (mine)
            __hip_atomic_store(halo_tile_flags(g_mb.peers[nbr(s)], par, s ^ 1) + flag_of(s), A.hx_epoch, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t t0 = wall_clock64();
        const bool ok = !mine || flag_wait(halo_tile_flags(g_mb.self, par, s) + flag_of(s), A.hx_epoch);
        const bool all = __all(ok);
        if (s == 0) {
            bx_ok = all ? 1 : 0;
            wait_note(kWaitHalo, t0);
        }
    }
    __syncthreads();
    if (!bx_ok) return false;
#pragma unroll
    for (int s = 0; s < kHaloSides; ++s) {
        if (!touches(s)) continue;
        const uint64_t* src = halo_inbox(g_mb.self, par, s, A.hx_cap);
        const int64_t base = s == 0 ? -pl : s == 1 ? nz * pl : s == 2 ? A.fy : s == 3 ? A.fy + nx * nz : s == 4 ? A.fx : A.fx + ny * nz;
        const int64_t len = plen(s);
        for (int64_t q = threadIdx.x; q < len; q += nthr) {
            int64_t f, unused;
            at(s, q, f, unused);
            v[base + f] = ld_inbox(src + f);
        }
    }
    __syncthreads();  // the march's loads of these layers follow (same workgroup)
    return true;
}

// ------------------------------------------------------------------------------ 3D stencil, LDS rows
// The same tile and z-march as k_st3d, but the y-neighbour rows come from the adjacent waves of the
// block through LDS: every wave cooks its own centre row of plane k (it already holds it for the z
// pipeline), stores it in a parity-double-buffered LDS row, and after one barrier per plane reads
// rows j +- 1 from there.  Only the tile's edge waves load a halo row (row j0 - 1 or j0 + NW, or the
// periodic wrap) -- per plane NW + 2 row loads per field instead of 3 NW, so taller tiles (NW = 8)
// cost no extra load issue and re-fetch (NW + 2) / NW of a plane instead of 1.5x.
// F0R: as k_st2d's -- F(u) recomputed from the u rows (and a second LDS row for the u field's
// y-neighbours) with the residual kernel's arithmetic instead of loading F0
// Waves per SIMD the 3D z-march is allocated for: 4 (<= 128 VGPRs instead of 132) for G_Euler!'s FD Jv + dot
// with F(u) recomputed -- the config-5 slab's Jv, 147 -> 141 us; every other instance unconstrained (the
// same cap on all of them: 512^3 Euler FD Jv 1160 -> 1257 us, midpoint 1303 -> 2900 us with spills,
// profiles/r04/ab_st3l_wpe.log)
#ifndef NK_ST3L_WPE
#define NK_ST3L_WPE(KIND, EPI, F0R, BLK) ((KIND == NK_HEAT3D_EULER && EPI == EPI_DOT && F0R && NK_ST3L_WPE_BLK(BLK)) ? 4 : 1)
#endif
#ifndef NK_ST3L_BLK_CAP  // (product variant build for A/B: 1 = the 4-wave cap for the BLK instance too)
#define NK_ST3L_BLK_CAP 0
#endif
#define NK_ST3L_WPE_BLK(BLK) (NK_ST3L_BLK_CAP || !(BLK))
// BLK (3D blocks, nk_dist_grid): the x / y ghost layers come from the faces after the allocation's trailing
// plane (KArgs::fy / fx, sides with a neighbour in KArgs::nbm) -- the left / right x-edges of the block's
// first / last column through the edge slots (the right one as the periodic wrap's second slot), the halo
// rows beyond the block's first / last row from the y faces; z keeps the ghost planes.
template <int KIND, int MODE, int EPI, int VEC, bool PER = false, int NW = 8, bool F0R = false, bool BLK = false>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NK_ST3L_WPE(KIND, EPI, F0R, BLK)))) void k_st3l(KArgs A0) {
    __shared__ double sh[kShN];
    const double* const et = nullptr;  // heat kinds: no exp
    bool rare_ = false;
    KArgs A = A0;
    if constexpr (!kKeepVdiv && EPI != EPI_DOTV && EPI != EPI_DOTVS) A.vdiv = nullptr;  // v / h only with V_k stored
    A.hd = A.vdiv ? *A.vdiv : 1.0;
    A.ihd = 1.0 / A.hd;
    constexpr int SCH = scheme_of<KIND>();
    constexpr bool kG = SCH != 0 && MODE != MODE_JEXACT;
    constexpr bool kTG = SCH == 2 && kG;  // G_Trapezoid!: u_n's y-neighbours too
    constexpr bool kR = MODE == MODE_JFD && F0R;
    __shared__ double ly[2][kTG ? 2 : 1][NW][64 * VEC];
    __shared__ double lyu[2][kR ? NW : 1][kR ? 64 * VEC : 1];  // F0R: the cooked u field's centre rows
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int nb = gridDim.x, b = blockIdx.x;
    int tz, txy;
    const int nzc = (int)((A.nz + A.rows - 1) / A.rows);
    if (BLK && A.torder) {  // the in-launch block exchange's order (host-built: exchanging tiles first)
        const int t = A.torder[b], tpl = A.tiles_x * A.tiles_y;
        tz = t / tpl;
        txy = t % tpl;
    } else {
        tile3_of(b, nb, A.tiles_x, A.tiles_y, nzc, A.hx_lo, A.hx_hi, A.zalt, tz, txy);
    }
    const int ty = txy / A.tiles_x, tx = txy % A.tiles_x;
    const int64_t nx = A.nx, ny = A.ny, nz = A.nz, pl = nx * ny;
    const int64_t x0 = (int64_t)tx * (64 * VEC) + (int64_t)lane * VEC;
    const int64_t j = (int64_t)ty * NW + wv;
    const bool act = x0 < nx && j < ny;
    const int64_t oj = (act ? j * nx + x0 : 0);
    constexpr bool kE2 = PER || BLK;  // the second x-edge slot: the periodic wrap, or a block's x-hi face
    // BLK: this lane's x-edges / this wave's halo rows from the faces (a neighbour on that side)
    const bool fxl = BLK && (A.nbm & 16) && lane == 0 && act && x0 == 0;
    const bool fxr = BLK && (A.nbm & 32) && act && x0 + VEC == nx;
    const bool fyn = BLK && (A.nbm & 8) && act && j + 1 == ny;
    const bool fys = BLK && (A.nbm & 4) && act && j == 0;
    // y-neighbours: from the adjacent wave's LDS row when it is in this tile, else a halo-row load
    const bool lds_n = wv + 1 < NW && j + 1 < ny;
    const bool lds_s = wv >= 1;
    bool has_n, has_s;
    int64_t dn_, ds;
    if constexpr (PER) {
        has_n = act;
        has_s = act;
        dn_ = !act ? 0 : (j + 1 < ny ? nx : -(ny - 1) * nx);
        ds = !act ? 0 : (j >= 1 ? -nx : (ny - 1) * nx);
    } else {
        has_n = act && (j + 1 < ny || fyn);
        has_s = act && (j >= 1 || fys);
        dn_ = has_n && !fyn ? nx : 0;
        ds = has_s && !fys ? -nx : 0;
    }
    const bool ld_n = !lds_n && has_n, ld_s = !lds_s && has_s;  // wave-uniform
    XEdge xe{};
    if constexpr (BLK) {  // in-array edges inside the block, faces at its x-ends -- one edge slot (one load per
        // field and row, as a slab's), the second only for a one-lane last tile's x-hi face (e2w, wave-uniform)
        const bool lin = lane == 0 && act && x0 >= 1, rin = lane == 63 && act && x0 + VEC < nx;
        xe.de = lin ? -1 : (rin ? VEC : 0);
        xe.ok = lin || fxl || rin || (fxr && lane != 0);
        xe.de2 = 0;
        xe.ok2 = fxr && lane == 0;
        xe.rwrap = fxr;
    } else {
        xe = x_edge<VEC, PER>(lane, act, x0, nx);
    }
    const int64_t de = xe.de, de2 = xe.de2;
    const bool edge_ok = xe.ok, edge_ok2 = xe.ok2;
    const int64_t z0 = (int64_t)tz * A.rows;
    const int64_t z1 = z0 + A.rows < nz ? z0 + A.rows : nz;
    // march direction: odd chunks (zalt) from z1 - 1 down to z0 -- fm / fp are then the planes above /
    // below, and the z-Laplacian takes them in the reference's order ((p - 2c) + m) all the same
#ifdef NK_KBENCH
    const bool dn = A.zalt && (tz & 1);
#else
    constexpr bool dn = false;  // the product keeps the plane-major order, upward marches (profiles/r03/ab_zalt2.log)
#endif
    const int64_t st = dn ? -pl : pl, dz = dn ? -1 : 1;
    const int64_t zs = dn ? z1 - 1 : z0;
    constexpr bool kUn = SCH == 0 && MODE != MODE_JEXACT;
    constexpr bool kF0 = MODE == MODE_JFD && !kR;
    constexpr bool kAx = EPI == EPI_DOT || EPI == EPI_DOTV || EPI == EPI_RESID;
    constexpr bool vout = MODE != MODE_RES && (EPI == EPI_DOTV || EPI == EPI_DOTVS);
    // ghost planes of v from the neighbours' patches, fetched by this launch (z-tiles at the slab's ends)
    const uint64_t* ib_lo = nullptr;
    const uint64_t* ib_hi = nullptr;
    if constexpr (MODE != MODE_RES && !PER && !BLK) {
        const HaloTile ht{A.hx_lo && z0 == 0 && z0 < nz, A.hx_hi && z1 == nz && z0 < nz};
        if (ht.lo || ht.hi) {  // block-uniform
            const int64_t ra = (int64_t)ty * NW, rb = ra + NW < ny ? ra + NW : ny;
            const int64_t ca = (int64_t)tx * (64 * VEC), cb = ca + 64 * VEC < nx ? ca + 64 * VEC : nx;
            if (halo_tile_exchange(A.v, pl, nz, nx, ra, rb, ca, cb, txy, ht, A.hx_epoch, A.hx_cap, 64 * NW)) {
                const int par = (int)(A.hx_epoch & 1);
                if (ht.lo) ib_lo = halo_inbox(g_mb.self, par, 0, A.hx_cap);
                if (ht.hi) ib_hi = halo_inbox(g_mb.self, par, 1, A.hx_cap);
            }
        }
    }
    if constexpr (MODE != MODE_RES && BLK) {
        if (A.hx_blk) (void)blk_tile_exchange<NW, VEC>(A, tx, ty, tz, z0, z1, nzc);  // (a time-out is flagged)
    }
    double acc = 0.0;
    // a plane ahead of the march (plane kk at offset o): the neighbour's patch from the inbox for a
    // ghost plane fetched in this launch, else memory
    // the x-edge offsets of plane kk (BLK: the faces for the block's end columns of an interior plane)
    auto eo1 = [&](int64_t kk, int64_t o) {
        if (BLK && kk >= 0 && kk < nz) {
            if (fxl) return A.fx + kk * ny + j;
            if (fxr && lane != 0) return A.fx + ny * nz + kk * ny + j;
        }
        return o + de;
    };
    auto eo2 = [&](int64_t kk, int64_t o) { return (fxr && kk >= 0 && kk < nz) ? A.fx + ny * nz + kk * ny + j : o + de2; };
    // BLK: the second edge slot's loads only where lane 0 is the x-hi face lane (a one-lane last tile)
    const bool e2w = !BLK || ((A.nbm & 32) && j < ny && (int64_t)tx * (64 * VEC) + VEC == nx);
    // the halo rows of plane kk beyond the tile (BLK: the y faces beyond the block's first / last row)
    auto nrow = [&](int64_t kk, int64_t o) { return fyn ? A.fy + nx * nz + kk * nx + x0 : o + dn_; };
    auto srow = [&](int64_t kk, int64_t o) { return fys ? A.fy + kk * nx + x0 : o + ds; };
    auto ahead = [&](int64_t kk, int64_t o) {
        const uint64_t* ib = (ib_hi && kk == nz) ? ib_hi : ((ib_lo && kk == -1) ? ib_lo : nullptr);
        return ib ? load_raw_ib<MODE, VEC, kG>(A, ib, o, oj) : load_raw<MODE, VEC, true, kG, kE2>(A, o, eo1(kk, o), eo2(kk, o), e2w);
    };
    if (z0 < nz) {
        const int64_t o0 = zs * pl + oj;
        const int64_t kb = zs - dz;  // the plane behind the first
        const uint64_t* ibb = (ib_lo && kb == -1) ? ib_lo : ((ib_hi && kb == nz) ? ib_hi : nullptr);
        const RawRow<MODE, VEC> rm0 =
            ibb ? load_raw_ib<MODE, VEC, kG>(A, ibb, o0 - st, oj) : load_raw<MODE, VEC, false, kG, kE2>(A, o0 - st, 0);
        const RawRow<MODE, VEC> rc0 = load_raw<MODE, VEC, true, kG, kE2>(A, o0, eo1(zs, o0), eo2(zs, o0), e2w);
        Field<VEC> fm = cook<MODE, VEC, SCH, kG, kE2>(A, rm0, act, false);
        Field<VEC> fc = cook<MODE, VEC, SCH, kG, kE2>(A, rc0, act, edge_ok, edge_ok2);
        Field<VEC> um{}, uc_{};  // F0R: the u field of planes k-1, k
        if constexpr (kR) {
            um = cook<MODE_RES, VEC, SCH, kG, kE2>(A, as_res_row<MODE, VEC>(rm0), act, false);
            uc_ = cook<MODE_RES, VEC, SCH, kG, kE2>(A, as_res_row<MODE, VEC>(rc0), act, edge_ok, edge_ok2);
        }
        RawRow<MODE, VEC> rp = ahead(zs + dz, o0 + st);
        RawRow<MODE, VEC> rn{}, rs{};
        if (ld_n) rn = load_raw<MODE, VEC, false, kG, kE2>(A, nrow(zs, o0), 0);
        if (ld_s) rs = load_raw<MODE, VEC, false, kG, kE2>(A, srow(zs, o0), 0);
        Row<VEC> unc{}, f0c{}, ax{};
        if constexpr (kUn) unc = data_row<VEC, NK_ST_NTN>(A.un, o0, true);
        if constexpr (kF0) f0c = data_row<VEC, NK_ST_NT>(A.F0, o0, true);
        if constexpr (kAx) ax = data_row<VEC>(A.aux, o0, true);
        const int cnt = (int)(z1 - z0);
        for (int it = 0; it < cnt; ++it) {
            const int64_t k = zs + it * dz;
            const int64_t o = k * pl + oj;
            const int par = it & 1;
            // ---- publish this wave's cooked centre row of plane k for its y-neighbours
#pragma unroll
            for (int q = 0; q < VEC; ++q) {
                ly[par][0][wv][lane * VEC + q] = fc.c[q];
                if constexpr (kTG) ly[par][kTG ? 1 : 0][wv][lane * VEC + q] = fc.g[q];
                if constexpr (kR) lyu[par][kR ? wv : 0][kR ? lane * VEC + q : 0] = uc_.c[q];
            }
            // ---- issue: centre row of plane k+2, halo rows and centre data of plane k+1
            const bool more = it + 1 < cnt;
            const int64_t o2 = more ? o + 2 * st : o + st;
            const int64_t o1 = more ? o + st : o;
            const int64_t k2 = more ? k + 2 * dz : k + dz;  // the plane o2 is in (-1 / nz: a ghost plane)
            const RawRow<MODE, VEC> rpp = ahead(k2, o2);
            RawRow<MODE, VEC> rnn{}, rss{};
            const int64_t k1 = more ? k + dz : k;  // the plane o1 is in
            if (ld_n) rnn = load_raw<MODE, VEC, false, kG, kE2>(A, nrow(k1, o1), 0);
            if (ld_s) rss = load_raw<MODE, VEC, false, kG, kE2>(A, srow(k1, o1), 0);
            Row<VEC> uncn{}, f0cn{}, axn{};
            if constexpr (kUn) uncn = data_row<VEC, NK_ST_NTN>(A.un, o1, true);
            if constexpr (kF0) f0cn = data_row<VEC, NK_ST_NT>(A.F0, o1, true);
            if constexpr (kAx) axn = data_row<VEC>(A.aux, o1, true);
            // ---- cook what was issued one iteration ago
            const Field<VEC> fp = cook<MODE, VEC, SCH, kG, kE2>(A, rp, act, edge_ok, edge_ok2);
            Field<VEC> fn{}, fs{};
            if (ld_n) fn = cook<MODE, VEC, SCH, kG, kE2>(A, rn, has_n, false);
            if (ld_s) fs = cook<MODE, VEC, SCH, kG, kE2>(A, rs, has_s, false);
            Field<VEC> up{}, fnu{}, fsu{};
            if constexpr (kR) {
                up = cook<MODE_RES, VEC, SCH, kG, kE2>(A, as_res_row<MODE, VEC>(rp), act, edge_ok, edge_ok2);
                if (ld_n) fnu = cook<MODE_RES, VEC, SCH, kG, kE2>(A, as_res_row<MODE, VEC>(rn), has_n, false);
                if (ld_s) fsu = cook<MODE_RES, VEC, SCH, kG, kE2>(A, as_res_row<MODE, VEC>(rs), has_s, false);
            }
            __syncthreads();  // plane k's rows are in LDS (parity: the next plane's writes go to the other buffer)
            double cn[VEC], cs[VEC], gn[VEC], gs[VEC];
#pragma unroll
            for (int q = 0; q < VEC; ++q) {
                cn[q] = lds_n ? ly[par][0][wv + (lds_n ? 1 : 0)][lane * VEC + q] : fn.c[q];
                cs[q] = lds_s ? ly[par][0][wv - (lds_s ? 1 : 0)][lane * VEC + q] : fs.c[q];
                if constexpr (kTG) {
                    gn[q] = lds_n ? ly[par][1][wv + (lds_n ? 1 : 0)][lane * VEC + q] : fn.g[q];
                    gs[q] = lds_s ? ly[par][1][wv - (lds_s ? 1 : 0)][lane * VEC + q] : fs.g[q];
                } else {
                    gn[q] = gs[q] = 0.0;
                }
                if (!has_n) { cn[q] = 0.0; gn[q] = 0.0; }  // bc_zero! beyond the last row
                if (!has_s) { cs[q] = 0.0; gs[q] = 0.0; }
            }
            double cnu[VEC], csu[VEC];  // F0R: the u field's y-neighbours
            LR xu{};
            if constexpr (kR) {
#pragma unroll
                for (int q = 0; q < VEC; ++q) {
                    cnu[q] = lds_n ? lyu[par][kR ? wv + (lds_n ? 1 : 0) : 0][kR ? lane * VEC + q : 0] : fnu.c[q];
                    csu[q] = lds_s ? lyu[par][kR ? wv - (lds_s ? 1 : 0) : 0][kR ? lane * VEC + q : 0] : fsu.c[q];
                    if (!has_n) cnu[q] = 0.0;
                    if (!has_s) csu[q] = 0.0;
                }
                xu = x_nbrs<kE2, BLK>(A, uc_.c[0], uc_.c[VEC - 1], uc_.e, uc_.e2, lane, xe.rwrap);
            }
            // ---- compute plane k
            const LR xn = x_nbrs<kE2, BLK>(A, fc.c[0], fc.c[VEC - 1], fc.e, fc.e2, lane, xe.rwrap);
            const double lft = xn.l, rgt = xn.r;
            double glft = 0.0, grgt = 0.0;
            if constexpr (SCH == 2 && kG) {
                const LR g2 = x_nbrs<kE2, BLK>(A, fc.g[0], fc.g[VEC - 1], fc.ge, fc.ge2, lane, xe.rwrap);
                glft = g2.l;
                grgt = g2.r;
            }
            if (act) {
                Row<VEC> val;
#pragma unroll
                for (int q = 0; q < VEC; ++q) {
                    const double w = (q == 0) ? lft : fc.c[q == 0 ? 0 : q - 1];
                    const double e = (q == VEC - 1) ? rgt : fc.c[q == VEC - 1 ? q : q + 1];
                    const double c = fc.c[q];
                    const double lsum = (lapk(A, c, e, w, A.hx2, A.ihx2) + lapk(A, c, cn[q], cs[q], A.hy2, A.ihy2)) +
                                        lapk(A, c, dn ? fm.c[q] : fp.c[q], dn ? fp.c[q] : fm.c[q], A.hz2, A.ihz2);
                    double lsumg = 0.0;
                    if constexpr (SCH == 2 && kG) {
                        const double g = fc.g[q];
                        const double gw = (q == 0) ? glft : fc.g[q == 0 ? 0 : q - 1];
                        const double ge = (q == VEC - 1) ? grgt : fc.g[q == VEC - 1 ? q : q + 1];
                        lsumg = (lapk(A, g, ge, gw, A.hx2, A.ihx2) + lapk(A, g, gn[q], gs[q], A.hy2, A.ihy2)) +
                                lapk(A, g, dn ? fm.g[q] : fp.g[q], dn ? fp.g[q] : fm.g[q], A.hz2, A.ihz2);
                    }
                    const double unq = kG ? fc.g[q] : unc.v[q];
                    double f0 = f0c.v[q];
                    if constexpr (kR) {  // F(u) at this point, as the residual kernel evaluates it
                        const double uw = (q == 0) ? xu.l : uc_.c[q == 0 ? 0 : q - 1];
                        const double ue = (q == VEC - 1) ? xu.r : uc_.c[q == VEC - 1 ? q : q + 1];
                        const double ucc = uc_.c[q];
                        const double lsu = (lapk(A, ucc, ue, uw, A.hx2, A.ihx2) + lapk(A, ucc, cnu[q], csu[q], A.hy2, A.ihy2)) +
                                           lapk(A, ucc, dn ? um.c[q] : up.c[q], dn ? up.c[q] : um.c[q], A.hz2, A.ihz2);
                        f0 = point_value<KIND, MODE_RES>(A, ucc, lsu, 0.0, unq, 0.0, SCH == 1 ? uc_.x[q] : ucc, lsumg, et, rare_);
                    }
                    double r = point_value<KIND, MODE>(A, c, lsum, 0.0, unq, f0, SCH == 1 ? fc.x[q] : c, lsumg, et, rare_);
                    acc = epilogue<EPI>(r, EPI == EPI_DOTVS ? fc.vn[q] : ax.v[q], acc);
                    val.v[q] = r;
                }
                store_row<VEC>(A.out, o, val);
                if (vout) {
                    Row<VEC> vn;
#pragma unroll
                    for (int q = 0; q < VEC; ++q) vn.v[q] = fc.vn[q];
                    store_row<VEC, NK_ST_NT>(A.vout, o, vn);
                }
            }
            fm = fc;
            fc = fp;
            if constexpr (kR) {
                um = uc_;
                uc_ = up;
            }
            rp = rpp;
            rn = rnn;
            rs = rss;
            unc = uncn;
            f0c = f0cn;
            ax = axn;
        }
    }
    if constexpr (EPI != EPI_NONE) publish<64 * NW>(acc, A.part, A.fin, sh, tz * A.tiles_x * A.tiles_y + txy);
}

// ------------------------------------------------------------------------------ stencil dispatch
// Every dispatch returns what it launched (StInst): the byte model, the F0R launch counters and the
// profile's kernel name are taken from the instantiation that ran, never from the policy flags.
inline const char* st_tf(bool b) { return b ? "true" : "false"; }

template <int MODE, int EPI>
StInst go_st1d(const KArgs& A, int grid, hipStream_t s) {
    hipLaunchKernelGGL((k_st1d<MODE, EPI>), dim3(grid), dim3(kBlock), 0, s, A);
    StInst r{};
    snprintf(r.name, sizeof r.name, "nk::k_st1d<%d, %d>", MODE, EPI);
    return r;
}

template <int KIND, int MODE, int EPI, int VEC, bool PER = false, bool F0R = false>
StInst go_st2d(const KArgs& A, int grid, hipStream_t s) {
    hipLaunchKernelGGL((k_st2d<KIND, MODE, EPI, VEC, PER, F0R>), dim3(grid), dim3(kBlock), 0, s, A);
    StInst r{};
    snprintf(r.name, sizeof r.name, "nk::k_st2d<%d, %d, %d, %d, %s, %s>", KIND, MODE, EPI, VEC, st_tf(PER), st_tf(F0R));
    r.f0r = F0R;
    return r;
}

template <int KIND, int MODE, int EPI, int VEC, bool PER, int NW, bool F0R, bool BLK = false>
StInst go_st3l_i(const KArgs& A, int grid, hipStream_t s) {
    hipLaunchKernelGGL((k_st3l<KIND, MODE, EPI, VEC, PER, NW, F0R, BLK>), dim3(grid), dim3(64 * NW), 0, s, A);
    StInst r{};
    snprintf(r.name, sizeof r.name, "nk::k_st3l<%d, %d, %d, %d, %s, %d, %s, %s>", KIND, MODE, EPI, VEC, st_tf(PER), NW,
             st_tf(F0R), st_tf(BLK));
    r.f0r = F0R;
    return r;
}

template <int KIND, int MODE, int EPI, int NW>
StInst go_st3l(const KArgs& A, int vec, int grid, hipStream_t s, bool per) {
#ifdef NK_KBENCH
    constexpr bool kF0R = MODE == MODE_JFD && heat_kind<KIND>();
#else
    constexpr bool kF0R = MODE == MODE_JFD && KIND == NK_HEAT3D_EULER;  // the only 3D F0R kind the launcher picks
#endif
    if (A.blk) {  // 3D blocks: bc_zero! only
        if constexpr (kF0R) {
            if (A.f0r) return vec == 2 ? go_st3l_i<KIND, MODE, EPI, 2, false, NW, true, true>(A, grid, s)
                                       : go_st3l_i<KIND, MODE, EPI, 1, false, NW, true, true>(A, grid, s);
        }
        return vec == 2 ? go_st3l_i<KIND, MODE, EPI, 2, false, NW, false, true>(A, grid, s)
                        : go_st3l_i<KIND, MODE, EPI, 1, false, NW, false, true>(A, grid, s);
    }
    if constexpr (kF0R) {  // F0 recomputed from u (KArgs::f0r)
        if (A.f0r) {
            if (per) return vec == 2 ? go_st3l_i<KIND, MODE, EPI, 2, true, NW, true>(A, grid, s)
                                     : go_st3l_i<KIND, MODE, EPI, 1, true, NW, true>(A, grid, s);
            return vec == 2 ? go_st3l_i<KIND, MODE, EPI, 2, false, NW, true>(A, grid, s)
                            : go_st3l_i<KIND, MODE, EPI, 1, false, NW, true>(A, grid, s);
        }
    }
    if (per) return vec == 2 ? go_st3l_i<KIND, MODE, EPI, 2, true, NW, false>(A, grid, s)
                             : go_st3l_i<KIND, MODE, EPI, 1, true, NW, false>(A, grid, s);
    return vec == 2 ? go_st3l_i<KIND, MODE, EPI, 2, false, NW, false>(A, grid, s)
                    : go_st3l_i<KIND, MODE, EPI, 1, false, NW, false>(A, grid, s);
}

}  // namespace
}  // namespace nk

#ifdef NK_KBENCH  // the variants only the kernel-variant bench build dispatches (tools/, DESIGN §4 no-gos)
#include "nk_stencil_var.hpp"
#endif

namespace nk {
namespace {

template <int KIND, int MODE, int EPI>
StInst go_stencil(const KArgs& A, int vec, int grid, hipStream_t s, bool per) {
    constexpr bool k2d = KIND == NK_BRATU2D || KIND == NK_HEAT2D_EULER || KIND == NK_HEAT2D_MIDPOINT ||
                         KIND == NK_HEAT2D_TRAPEZOID;
    if constexpr (KIND == NK_BRATU1D) {
        return go_st1d<MODE, EPI>(A, grid, s);
    } else if constexpr (k2d) {
#ifdef NK_KBENCH
        // one-shot LDS tiles (k_st2t, kernel-variant build only: NK_ST_ONESHOT / fast bits)
        if (A.tile2) return go_st2t<KIND, MODE, EPI>(A, vec, grid, s, per);
#endif
        if constexpr (MODE == MODE_JFD) {  // F0 recomputed from u (KArgs::f0r), VEC <= 2
            if (A.f0r && vec <= 2) {
                if constexpr (heat_kind<KIND>()) {  // bc_periodic! (heat only) with F(u) recomputed
                    if (per) return vec == 2 ? go_st2d<KIND, MODE, EPI, 2, true, true>(A, grid, s)
                                             : go_st2d<KIND, MODE, EPI, 1, true, true>(A, grid, s);
                }
                return vec == 2 ? go_st2d<KIND, MODE, EPI, 2, false, true>(A, grid, s)
                                : go_st2d<KIND, MODE, EPI, 1, false, true>(A, grid, s);
            }
        }
        if constexpr (heat_kind<KIND>()) {  // bc_periodic! instantiations: heat only, VEC <= 2
            if (per) return vec == 2 ? go_st2d<KIND, MODE, EPI, 2, true>(A, grid, s)
                                     : go_st2d<KIND, MODE, EPI, 1, true>(A, grid, s);
        }
#ifdef NK_KBENCH
        if (vec == 4) return go_st2d<KIND, MODE, EPI, 4>(A, grid, s);
#endif
        return vec == 2 ? go_st2d<KIND, MODE, EPI, 2>(A, grid, s) : go_st2d<KIND, MODE, EPI, 1>(A, grid, s);
    } else {
        // k_st3l: y-neighbours through LDS, 4-row tiles (the kernel-variant build: 8-row tiles, the
        // per-wave y-row loads of k_st3d, the y-march k_st3y)
#ifdef NK_KBENCH
        if (!A.blk) {  // (3D blocks: k_st3l with 4-row tiles only)
            if (A.ym) return A.nw == 8 ? go_st3y<KIND, MODE, EPI, 8>(A, vec, grid, s, per)
                                       : go_st3y<KIND, MODE, EPI, 4>(A, vec, grid, s, per);
            if (!A.lds3) return go_st3d<KIND, MODE, EPI, 4>(A, vec, grid, s, per);
            if (A.nw == 8) return go_st3l<KIND, MODE, EPI, 8>(A, vec, grid, s, per);
        }
#endif
        return go_st3l<KIND, MODE, EPI, 4>(A, vec, grid, s, per);
    }
}

template <int KIND, int MODE>
StInst go_stencil_epi(const KArgs& A, int epi, int vec, int grid, hipStream_t s, bool per) {
    switch (epi) {
    case EPI_NONE: return go_stencil<KIND, MODE, EPI_NONE>(A, vec, grid, s, per);
    case EPI_SUMSQ: return go_stencil<KIND, MODE, EPI_SUMSQ>(A, vec, grid, s, per);
    case EPI_DOT: return go_stencil<KIND, MODE, EPI_DOT>(A, vec, grid, s, per);
    case EPI_DOTV: return go_stencil<KIND, MODE, EPI_DOTV>(A, vec, grid, s, per);
    case EPI_DOTVS: return go_stencil<KIND, MODE, EPI_DOTVS>(A, vec, grid, s, per);
    default: return go_stencil<KIND, MODE, EPI_RESID>(A, vec, grid, s, per);
    }
}

template <int KIND>
StInst go_stencil_mode(const KArgs& A, int mode, int epi, int vec, int grid, hipStream_t s, bool per) {
    switch (mode) {
    case MODE_RES: return go_stencil_epi<KIND, MODE_RES>(A, epi, vec, grid, s, per);
    case MODE_JEXACT: return go_stencil_epi<KIND, MODE_JEXACT>(A, epi, vec, grid, s, per);
    default: return go_stencil_epi<KIND, MODE_JFD>(A, epi, vec, grid, s, per);
    }
}

}  // namespace
}  // namespace nk
