// nk_stencil_kern.hpp -- the stencil kernel templates and their compile-time dispatch: the 2D row march
// (k_st2d), the 3D z-march with LDS rows (k_st3l, with the 3D blocks' faces and the opt-in in-launch face
// exchange blk_tile_exchange), go_stencil_mode.  Included by the per-kind instantiation units
// (nk_stencil_inst.hip) only; the shared pieces (KArgs, point_value, row loads, edges, tile order) are
// nk_stencil.hpp.
#pragma once
#include "nk_stencil.hpp"

namespace nk {
namespace {

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
        for (int64_t q0 = threadIdx.x; q0 < len; q0 += (int64_t)kXchgRoundBlk * nthr) {  // rounds: loads, one wait, stores
            double a[kXchgRoundBlk];
            int64_t f[kXchgRoundBlk];
#pragma unroll
            for (int r = 0; r < kXchgRoundBlk; ++r) {
                const int64_t q = q0 + (int64_t)r * nthr;
                int64_t src;
                at(s, q, f[r], src);
                a[r] = q < len ? v[src] : 0.0;
            }
            wait_loads();
#pragma unroll
            for (int r = 0; r < kXchgRoundBlk; ++r)
                if (q0 + (int64_t)r * nthr < len)
                    __hip_atomic_store(dst + f[r], (uint64_t)__double_as_longlong(a[r]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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
        for (int64_t q0 = threadIdx.x; q0 < len; q0 += (int64_t)kXchgRoundBlk * nthr) {
            double a[kXchgRoundBlk];
            int64_t f[kXchgRoundBlk];
#pragma unroll
            for (int r = 0; r < kXchgRoundBlk; ++r) {
                const int64_t q = q0 + (int64_t)r * nthr;
                int64_t unused;
                at(s, q, f[r], unused);
                a[r] = q < len ? ld_inbox(src + f[r]) : 0.0;
            }
            wait_loads();
#pragma unroll
            for (int r = 0; r < kXchgRoundBlk; ++r)
                if (q0 + (int64_t)r * nthr < len) v[base + f[r]] = a[r];
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
            if (halo_tile_exchange<1>(A.v, pl, nz, nx, ra, rb, ca, cb, txy, ht, A.hx_epoch, A.hx_cap, 64 * NW)) {
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
