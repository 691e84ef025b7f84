// nk_stencil_var.hpp -- stencil variants of the kernel-variant bench build only (lib/libnkhip_kbench.so,
// -DNK_KBENCH): measured against the product kernels of nk_stencil.hpp and not shipped:
//   k_st2t  2D one-shot LDS tiles (no march)         -- faster in isolation, not in the bench (r03)
//   k_st3d  3D z-march, y-neighbour rows per wave      -- k_st3l (LDS rows) is 6-16 % faster (r02)
//   k_st3y  3D y-march for slabs short along z         -- slower on every shape (r04)
// Included by nk_stencil.hpp after the shared helpers and k_st3l, before the dispatch.
#pragma once

namespace nk {
namespace {

// ------------------------------------------------------------------------------ 2D stencil, one-shot LDS tile
// Block = NW waves = NW rows x 64*VEC columns, no march: every wave loads and cooks ITS row once (the
// first / last wave also the tile's halo rows), publishes the cooked stencil field to LDS, and after
// one barrier computes its row with the y-neighbours from LDS, the x-neighbours by shuffles.  Tiles in
// address order: the grid sweeps the arrays front to back like a one-shot copy (the access shape the
// march lacks: 128 row bands streaming 2 MB apart), with (NW + 2) / NW loads and cooks per row.
template <int KIND, int MODE, int EPI, int VEC, bool PER = false, bool F0R = false, int NW = 8>
__global__ __launch_bounds__(64 * NW) void k_st2t(KArgs A0) {
    __shared__ double sh[kShN];
    NK_EXP_LDS(KIND)
    bool rare_ = false;
    KArgs A = A0;
    if constexpr (!kKeepVdiv && EPI != EPI_DOTV && EPI != EPI_DOTVS) A.vdiv = nullptr;  // v / h only with V_k stored
    A.hd = A.vdiv ? *A.vdiv : 1.0;
    A.ihd = 1.0 / A.hd;
    constexpr int SCH = scheme_of<KIND>();
    constexpr bool kG = SCH != 0 && MODE != MODE_JEXACT;
    constexpr bool kTG = SCH == 2 && kG;              // G_Trapezoid!: u_n's Laplacian
    constexpr bool kR = MODE == MODE_JFD && F0R;       // F0R: the u field as the residual kernel cooks it
    constexpr int W = 64 * VEC;
    __shared__ double lc[NW + 2][W];
    __shared__ double lg[kTG ? NW + 2 : 1][kTG ? W : 1];
    __shared__ double lu[kR ? NW + 2 : 1][kR ? W : 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // tiles in address order; with ghost rows inside the launch the slab-end row bands first (tile_of)
    const int t = tile_of(blockIdx.x, gridDim.x, A.tiles_x, A.tiles_y, A.hx_lo, A.hx_hi, 1);
    const int tx = t % A.tiles_x, ty = t / A.tiles_x;
    const int64_t nx = A.nx, ny = A.ny;
    const int64_t x0 = (int64_t)tx * W + (int64_t)lane * VEC;
    const bool act = x0 < nx;
    const int64_t xc = act ? x0 : 0;
    const XEdge xe = x_edge<VEC, PER>(lane, act, x0, nx);
    const int64_t de = xe.de, de2 = xe.de2;
    const bool edge_ok = xe.ok, edge_ok2 = xe.ok2;
    const int64_t y0 = (int64_t)ty * NW;
    const int64_t j = y0 + wv;                          // this wave's row
    constexpr bool kU = MODE == MODE_JEXACT && KIND == NK_BRATU2D;
    constexpr bool kUn = KIND == NK_HEAT2D_EULER && MODE != MODE_JEXACT;
    constexpr bool kF0 = MODE == MODE_JFD && !F0R;
    constexpr bool kAx = EPI == EPI_DOT || EPI == EPI_DOTV || EPI == EPI_RESID;
    constexpr bool vout = MODE != MODE_RES && (EPI == EPI_DOTV || EPI == EPI_DOTVS);
    // the rows this block's LDS holds: y0 - 1 .. y0 + NW (capped at ny, the upper ghost row)
    const bool own = j <= ny;                           // row ny (ghost) only as a neighbour
    const bool lo_halo = wv == 0, hi_halo = wv == NW - 1 && y0 + NW <= ny;
    // ghost rows of v from the neighbours' patches, fetched by this launch (row bands at the slab's ends)
    const uint64_t* ib_lo = nullptr;
    const uint64_t* ib_hi = nullptr;
    if constexpr (MODE != MODE_RES && !PER) {
        const HaloTile ht{A.hx_lo && y0 == 0, A.hx_hi && y0 + NW >= ny && y0 < ny};
        if (ht.lo || ht.hi) {  // block-uniform
            const int64_t ca = (int64_t)tx * W, cb = ca + W < nx ? ca + W : nx;
            if (halo_tile_exchange(A.v, nx, ny, nx, 0, 1, ca, cb, tx, ht, A.hx_epoch, A.hx_cap, 64 * NW)) {
                const int par = (int)(A.hx_epoch & 1);
                if (ht.lo) ib_lo = halo_inbox(g_mb.self, par, 0, A.hx_cap);
                if (ht.hi) ib_hi = halo_inbox(g_mb.self, par, 1, A.hx_cap);
            }
        }
    }
    auto raw_of = [&](int64_t r) {
        const int64_t o = r * nx + xc;
        return load_raw<MODE, VEC, true, kG, PER, NK_ST_NTU>(A, o, o + de, o + de2);
    };
    auto put = [&](int i, const RawRow<MODE, VEC>& r, bool eok, bool eok2, Field<VEC>* keep, Field<VEC>* keepu) {
        const Field<VEC> f = cook<MODE, VEC, SCH, kG, PER>(A, r, act, eok, eok2);
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            lc[i][lane * VEC + k] = f.c[k];
            if constexpr (kTG) lg[kTG ? i : 0][kTG ? lane * VEC + k : 0] = f.g[k];
        }
        if (keep) *keep = f;
        if constexpr (kR) {
            const Field<VEC> fu = cook<MODE_RES, VEC, SCH, kG, PER>(A, as_res_row<MODE, VEC>(r), act, eok, eok2);
#pragma unroll
            for (int k = 0; k < VEC; ++k) lu[kR ? i : 0][kR ? lane * VEC + k : 0] = fu.c[k];
            if (keepu) *keepu = fu;
        }
    };
    // ---- issue every load of this wave up front
    RawRow<MODE, VEC> rown{}, rlo{}, rhi{};
    if (own) rown = raw_of(j);
    if (lo_halo) rlo = raw_of(y0 - 1);
    if (hi_halo) rhi = raw_of(y0 + NW);
    // the slab-end tiles of an in-launch exchange: the ghost row (-1 / ny) comes from the inbox instead
    // (kept out of the loads above: a per-load branch there serialises their issue)
    if (ib_lo && lo_halo) rlo = load_raw_ib<MODE, VEC, kG>(A, ib_lo, -nx + xc, xc);
    if (ib_hi) {
        if (own && j == ny) rown = load_raw_ib<MODE, VEC, kG>(A, ib_hi, ny * nx + xc, xc);
        if (hi_halo && y0 + NW == ny) rhi = load_raw_ib<MODE, VEC, kG>(A, ib_hi, ny * nx + xc, xc);
    }
    Row<VEC> uc{}, unc{}, f0c{}, ax{};
    const bool comp = j < ny;
    if (comp) {
        const int64_t o = j * nx + xc;
        if constexpr (kU) uc = data_row<VEC>(A.u, o, true);
        if constexpr (kUn) unc = data_row<VEC, NK_ST_NTN>(A.un, o, true);
        if constexpr (kF0) f0c = data_row<VEC, NK_ST_NT>(A.F0, o, true);
        if constexpr (kAx) ax = data_row<VEC>(A.aux, o, true);
    }
    // ---- cook into LDS
    Field<VEC> fc{}, uc_{};
    if (own) put(wv + 1, rown, edge_ok && comp, edge_ok2 && comp, &fc, &uc_);
    if (lo_halo) put(0, rlo, false, false, nullptr, nullptr);
    if (hi_halo) put(NW + 1, rhi, false, false, nullptr, nullptr);
    __syncthreads();
    double acc = 0.0;
    if (comp && act) {
        const LR xn = x_nbrs<PER>(A, fc.c[0], fc.c[VEC - 1], fc.e, fc.e2, lane, xe.rwrap);
        LR gn{}, un_{};
        if constexpr (kTG) gn = x_nbrs<PER>(A, fc.g[0], fc.g[VEC - 1], fc.ge, fc.ge2, lane, xe.rwrap);
        if constexpr (kR) un_ = x_nbrs<PER>(A, uc_.c[0], uc_.c[VEC - 1], uc_.e, uc_.e2, lane, xe.rwrap);
        Row<VEC> val;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const int q = lane * VEC + k;
            const double w = (k == 0) ? xn.l : fc.c[k == 0 ? 0 : k - 1];
            const double e = (k == VEC - 1) ? xn.r : fc.c[k == VEC - 1 ? k : k + 1];
            const double c = fc.c[k];
            const double lsum = lapk(A, c, e, w, A.hx2, A.ihx2) + lapk(A, c, lc[wv + 2][q], lc[wv][q], A.hy2, A.ihy2);
            double lsumg = 0.0;
            if constexpr (kTG) {
                const double gw = (k == 0) ? gn.l : fc.g[k == 0 ? 0 : k - 1];
                const double ge = (k == VEC - 1) ? gn.r : fc.g[k == VEC - 1 ? k : k + 1];
                lsumg = lapk(A, fc.g[k], ge, gw, A.hx2, A.ihx2) +
                        lapk(A, fc.g[k], lg[kTG ? wv + 2 : 0][kTG ? q : 0], lg[kTG ? wv : 0][kTG ? q : 0], A.hy2, A.ihy2);
            }
            const double unk = kG ? fc.g[k] : unc.v[k];
            double f0 = f0c.v[k];
            if constexpr (kR) {
                const double uw = (k == 0) ? un_.l : uc_.c[k == 0 ? 0 : k - 1];
                const double ue = (k == VEC - 1) ? un_.r : uc_.c[k == VEC - 1 ? k : k + 1];
                const double ucc = uc_.c[k];
                const double lsu = lapk(A, ucc, ue, uw, A.hx2, A.ihx2) +
                                   lapk(A, ucc, lu[kR ? wv + 2 : 0][kR ? q : 0], lu[kR ? wv : 0][kR ? q : 0], A.hy2, A.ihy2);
                f0 = point_value<KIND, MODE_RES>(A, ucc, lsu, 0.0, unk, 0.0, SCH == 1 ? uc_.x[k] : ucc, lsumg, et, rare_);
            }
            double r = point_value<KIND, MODE>(A, c, lsum, uc.v[k], unk, f0, SCH == 1 ? fc.x[k] : c, lsumg, et, rare_);
            acc = epilogue<EPI>(r, EPI == EPI_DOTVS ? fc.vn[k] : ax.v[k], acc);
            val.v[k] = r;
        }
        const int64_t o = j * nx + xc;
        store_row<VEC>(A.out, o, val);
        if (vout) {
            Row<VEC> vn;
#pragma unroll
            for (int k = 0; k < VEC; ++k) vn.v[k] = fc.vn[k];
            store_row<VEC, NK_ST_NT>(A.vout, o, vn);
        }
    }
    if constexpr (EPI != EPI_NONE) {
        if (A.group > 1) {  // per-tile partial; k_tile_fold hands on the group sums
            const double bs = block_sum<64 * NW>(acc, sh);
            if (threadIdx.x == 0) A.tpart[t] = bs;
        } else {
            publish<64 * NW>(acc, A.part, A.fin, sh, t);
        }
    }
}

// ------------------------------------------------------------------------------ 3D stencil
// Block = NW waves = NW rows (y) x 64*VEC columns, marching A.rows planes in z (NW = A.nw: taller
// tiles re-fetch fewer y-halo rows).  Same pipeline as
// the 2D kernel: at iteration k the raw loads of the centre row of plane k+2 and of the y-
// neighbour rows of plane k+1 are issued, plane k+1's centre row and plane k's y-neighbours
// (issued one iteration earlier) are cooked, and plane k is computed from registers.  The y-
// neighbour rows are mostly L2 hits (the adjacent waves of the block stream them).  PER: the
// y-neighbours of rows 0 and ny-1 wrap (bc_periodic!), x as in the 2D kernel.
template <int KIND, int MODE, int EPI, int VEC, bool PER = false, int NW = 4>
__global__ __launch_bounds__(64 * NW) void k_st3d(KArgs A0) {
    __shared__ double sh[kShN];
    const double* const et = nullptr;  // heat kinds: no exp
    bool rare_ = false;
    KArgs A = A0;
    if constexpr (!kKeepVdiv && EPI != EPI_DOTV && EPI != EPI_DOTVS) A.vdiv = nullptr;  // v / h only with V_k stored
    A.hd = A.vdiv ? *A.vdiv : 1.0;
    A.ihd = 1.0 / A.hd;
    constexpr int SCH = scheme_of<KIND>();
    constexpr bool kG = SCH != 0 && MODE != MODE_JEXACT;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int nb = gridDim.x, b = blockIdx.x;
    const int t = (nb & 7) == 0 ? (b & 7) * (nb >> 3) + (b >> 3) : b;
    const int tpl = A.tiles_x * A.tiles_y;
    const int tz = t / tpl, txy = t % tpl;
    const int ty = txy / A.tiles_x, tx = txy % A.tiles_x;
    const int64_t nx = A.nx, ny = A.ny, nz = A.nz, pl = nx * ny;
    const int64_t x0 = (int64_t)tx * (64 * VEC) + (int64_t)lane * VEC;
    const int64_t j = (int64_t)ty * NW + wv;
    const bool act = x0 < nx && j < ny;
    const int64_t oj = (act ? j * nx + x0 : 0);  // clamped: every load stays inside the allocation
    bool has_n, has_s;
    int64_t dn, ds;  // 0: dummy (own row), cooked to zero
    if constexpr (PER) {
        has_n = act;
        has_s = act;
        dn = !act ? 0 : (j + 1 < ny ? nx : -(ny - 1) * nx);
        ds = !act ? 0 : (j >= 1 ? -nx : (ny - 1) * nx);
    } else {
        has_n = act && j + 1 < ny;
        has_s = act && j >= 1;
        dn = has_n ? nx : 0;
        ds = has_s ? -nx : 0;
    }
    const XEdge xe = x_edge<VEC, PER>(lane, act, x0, nx);
    const int64_t de = xe.de, de2 = xe.de2;
    const bool edge_ok = xe.ok, edge_ok2 = xe.ok2;
    const int64_t z0 = (int64_t)tz * A.rows;
    const int64_t z1 = z0 + A.rows < nz ? z0 + A.rows : nz;
    constexpr bool kUn = SCH == 0 && MODE != MODE_JEXACT;
    constexpr bool kF0 = MODE == MODE_JFD;
    constexpr bool kAx = EPI == EPI_DOT || EPI == EPI_DOTV || EPI == EPI_RESID;
    constexpr bool vout = MODE != MODE_RES && (EPI == EPI_DOTV || EPI == EPI_DOTVS);  // fused kdivcopy!: V_k stored
    double acc = 0.0;
    if (z0 < nz) {
        const int64_t o0 = z0 * pl + oj;
        Field<VEC> fm = cook<MODE, VEC, SCH, kG, PER>(A, load_raw<MODE, VEC, false, kG, PER>(A, o0 - pl, 0), act, false);  // plane -1: ghost
        Field<VEC> fc = cook<MODE, VEC, SCH, kG, PER>(A, load_raw<MODE, VEC, true, kG, PER>(A, o0, o0 + de, o0 + de2), act,
                                                      edge_ok, edge_ok2);
        RawRow<MODE, VEC> rp = load_raw<MODE, VEC, true, kG, PER>(A, o0 + pl, o0 + pl + de, o0 + pl + de2);  // plane nz: ghost
        RawRow<MODE, VEC> rn = load_raw<MODE, VEC, false, kG, PER>(A, o0 + dn, 0);
        RawRow<MODE, VEC> rs = load_raw<MODE, VEC, false, kG, PER>(A, o0 + ds, 0);
        Row<VEC> unc{}, f0c{}, ax{};
        if constexpr (kUn) unc = data_row<VEC, NK_ST_NTN>(A.un, o0, true);
        if constexpr (kF0) f0c = data_row<VEC, NK_ST_NT>(A.F0, o0, true);
        if constexpr (kAx) ax = data_row<VEC>(A.aux, o0, true);
        for (int64_t k = z0; k < z1; ++k) {
            const int64_t o = k * pl + oj;
            // ---- issue: centre row of plane k+2, y-neighbour rows and centre data of plane k+1
            const bool more = k + 1 < z1;
            const int64_t o2 = more ? o + 2 * pl : o + pl;
            const int64_t o1 = more ? o + pl : o;
            const RawRow<MODE, VEC> rpp = load_raw<MODE, VEC, true, kG, PER>(A, o2, o2 + de, o2 + de2);
            const RawRow<MODE, VEC> rnn = load_raw<MODE, VEC, false, kG, PER>(A, o1 + dn, 0);
            const RawRow<MODE, VEC> rss = load_raw<MODE, VEC, false, kG, PER>(A, o1 + ds, 0);
            Row<VEC> uncn{}, f0cn{}, axn{};
            if constexpr (kUn) uncn = data_row<VEC, NK_ST_NTN>(A.un, o1, true);
            if constexpr (kF0) f0cn = data_row<VEC, NK_ST_NT>(A.F0, o1, true);
            if constexpr (kAx) axn = data_row<VEC>(A.aux, o1, true);
            // ---- cook what was issued one iteration ago
            const Field<VEC> fp = cook<MODE, VEC, SCH, kG, PER>(A, rp, act, edge_ok, edge_ok2);
            const Field<VEC> fn = cook<MODE, VEC, SCH, kG, PER>(A, rn, has_n, false);
            const Field<VEC> fs = cook<MODE, VEC, SCH, kG, PER>(A, rs, has_s, false);
            // ---- compute plane k
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
                for (int q = 0; q < VEC; ++q) {
                    const double w = (q == 0) ? lft : fc.c[q == 0 ? 0 : q - 1];
                    const double e = (q == VEC - 1) ? rgt : fc.c[q == VEC - 1 ? q : q + 1];
                    const double c = fc.c[q];
                    const double lsum = (lapk(A, c, e, w, A.hx2, A.ihx2) + lapk(A, c, fn.c[q], fs.c[q], A.hy2, A.ihy2)) +
                                        lapk(A, c, fp.c[q], fm.c[q], A.hz2, A.ihz2);
                    double lsumg = 0.0;
                    if constexpr (SCH == 2 && kG) {
                        const double g = fc.g[q];
                        const double gw = (q == 0) ? glft : fc.g[q == 0 ? 0 : q - 1];
                        const double ge = (q == VEC - 1) ? grgt : fc.g[q == VEC - 1 ? q : q + 1];
                        lsumg = (lapk(A, g, ge, gw, A.hx2, A.ihx2) + lapk(A, g, fn.g[q], fs.g[q], A.hy2, A.ihy2)) +
                                lapk(A, g, fp.g[q], fm.g[q], A.hz2, A.ihz2);
                    }
                    const double unq = kG ? fc.g[q] : unc.v[q];
                    double r = point_value<KIND, MODE>(A, c, lsum, 0.0, unq, f0c.v[q], SCH == 1 ? fc.x[q] : c, lsumg, et, rare_);
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
            rp = rpp;
            rn = rnn;
            rs = rss;
            unc = uncn;
            f0c = f0cn;
            ax = axn;
        }
    }
    if constexpr (EPI != EPI_NONE) publish<64 * NW>(acc, A.part, A.fin, sh);
}

// ------------------------------------------------------------------------------ 3D stencil, y-march
// For slabs that are short along z (config 5: 512^2 x 64 per rank): the tile is NW consecutive PLANES
// (one wave each) x 64*VEC columns, and it marches along y over a chunk of A.rows rows.  The roles of
// k_st3l's axes swap: the z-neighbours of row j come from the adjacent waves through LDS (the tile's
// edge waves load the halo planes' row -- the slab's ghost planes from memory, or from the inbox when
// they travel in this launch), the y-neighbours are the march's registers, x-neighbours shuffles.  The
// march re-reads (rows + 2) / rows of each field instead of the z-march's (16 + 2) / 16.  Arithmetic and
// association order are k_st3l's: ((x-Laplacian + y-Laplacian) + z-Laplacian), so every output is
// bit-identical to it.  Rows -1 / ny are not in memory (the ghost layer lives along z only): the zero
// boundary there, or the wrapped row under bc_periodic!.
template <int KIND, int MODE, int EPI, int VEC, bool PER = false, int NW = 4, bool F0R = false>
__global__ __launch_bounds__(64 * NW) void k_st3y(KArgs A0) {
    __shared__ double sh[kShN];
    const double* const et = nullptr;  // heat kinds: no exp
    bool rare_ = false;
    KArgs A = A0;
    if constexpr (!kKeepVdiv && EPI != EPI_DOTV && EPI != EPI_DOTVS) A.vdiv = nullptr;  // v / h only with V_k stored
    A.hd = A.vdiv ? *A.vdiv : 1.0;
    A.ihd = 1.0 / A.hd;
    constexpr int SCH = scheme_of<KIND>();
    constexpr bool kG = SCH != 0 && MODE != MODE_JEXACT;
    constexpr bool kTG = SCH == 2 && kG;
    constexpr bool kR = MODE == MODE_JFD && F0R;
    __shared__ double lz[2][kTG ? 2 : 1][NW][64 * VEC];
    __shared__ double lzu[2][kR ? NW : 1][kR ? 64 * VEC : 1];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int nb = gridDim.x, b = blockIdx.x;
    const int64_t nx = A.nx, ny = A.ny, nz = A.nz, pl = nx * ny;
    int tz, txy;
    tile3_of(b, nb, A.tiles_x, A.tiles_y, (int)((nz + NW - 1) / NW), A.hx_lo, A.hx_hi, 0, tz, txy);
    const int ty = txy / A.tiles_x, tx = txy % A.tiles_x;
    const int64_t x0 = (int64_t)tx * (64 * VEC) + (int64_t)lane * VEC;
    const int64_t k = (int64_t)tz * NW + wv;  // my plane
    const bool act = x0 < nx && k < nz;
    const int64_t ok0 = act ? k * pl + x0 : 0;  // row 0 of my plane at my columns
    // z-neighbours: the adjacent wave's LDS row when it is in this tile, else the halo plane's row (the
    // ghost planes -1 / nz exist in memory: zero, or the neighbour slab's / the ring's plane)
    const bool lds_u = wv + 1 < NW && k + 1 < nz;
    const bool lds_d = wv >= 1;
    const bool ld_u = !lds_u && act, ld_d = !lds_d && act;  // wave-uniform
    const XEdge xe = x_edge<VEC, PER>(lane, act, x0, nx);
    const int64_t de = xe.de, de2 = xe.de2;
    const bool edge_ok = xe.ok, edge_ok2 = xe.ok2;
    const int64_t y0 = (int64_t)ty * A.rows;
    const int64_t y1 = y0 + A.rows < ny ? y0 + A.rows : ny;
    constexpr bool kUn = SCH == 0 && MODE != MODE_JEXACT;
    constexpr bool kF0 = MODE == MODE_JFD && !kR;
    constexpr bool kAx = EPI == EPI_DOT || EPI == EPI_DOTV || EPI == EPI_RESID;
    constexpr bool vout = MODE != MODE_RES && (EPI == EPI_DOTV || EPI == EPI_DOTVS);
    // ghost planes of v fetched in this launch: the z-tiles at the slab's ends exchange the patch rows
    // [y0, y1) x their columns of my first / last plane
    const uint64_t* ib_lo = nullptr;
    const uint64_t* ib_hi = nullptr;
    if constexpr (MODE != MODE_RES && !PER) {
        const int nzt = (int)((nz + NW - 1) / NW);
        const HaloTile ht{A.hx_lo && tz == 0 && y0 < ny, A.hx_hi && tz == nzt - 1 && y0 < ny};
        if (ht.lo || ht.hi) {  // block-uniform
            const int64_t ca = (int64_t)tx * (64 * VEC), cb = ca + 64 * VEC < nx ? ca + 64 * VEC : nx;
            if (halo_tile_exchange(A.v, pl, nz, nx, y0, y1, ca, cb, txy, ht, A.hx_epoch, A.hx_cap, 64 * NW)) {
                const int par = (int)(A.hx_epoch & 1);
                if (ht.lo) ib_lo = halo_inbox(g_mb.self, par, 0, A.hx_cap);
                if (ht.hi) ib_hi = halo_inbox(g_mb.self, par, 1, A.hx_cap);
            }
        }
    }
    // the inbox holding my halo plane's row, if any (wave-uniform)
    const uint64_t* ibu = (ib_hi && k + 1 == nz) ? ib_hi : nullptr;
    const uint64_t* ibd = (ib_lo && k == 0) ? ib_lo : nullptr;
    // row r of my plane (r in [-1, ny]): in range, or wrapped (PER); rows -1 / ny are zero otherwise
    auto row_ok = [&](int64_t r) { return PER || (r >= 0 && r < ny); };
    auto row_off = [&](int64_t r) {
        const int64_t rr = PER ? (r < 0 ? r + ny : (r >= ny ? r - ny : r)) : (r < 0 ? 0 : (r >= ny ? ny - 1 : r));
        return ok0 + rr * nx;
    };
    auto centre_row = [&](int64_t r) {
        const int64_t o = row_off(r);
        return load_raw<MODE, VEC, true, kG, PER>(A, o, o + de, o + de2);
    };
    auto halo_row = [&](int64_t r, bool up) {  // plane k +- 1, row r (r in [0, ny))
        const int64_t o = row_off(r) + (up ? pl : -pl);
        const uint64_t* ib = up ? ibu : ibd;
        return ib ? load_raw_ib<MODE, VEC, kG>(A, ib, o, o - (up ? (k + 1) : (k - 1)) * pl)
                  : load_raw<MODE, VEC, false, kG, PER>(A, o, 0);
    };
    double acc = 0.0;
    if (y0 < ny && tz * (int64_t)NW < nz) {
        // rows y0-1 and y0 cooked up front; row y0+1 raw in flight
        const RawRow<MODE, VEC> rm0 = centre_row(y0 - 1);
        const RawRow<MODE, VEC> rc0 = centre_row(y0);
        Field<VEC> fm = cook<MODE, VEC, SCH, kG, PER>(A, rm0, act && row_ok(y0 - 1), edge_ok && row_ok(y0 - 1),
                                                      edge_ok2 && row_ok(y0 - 1));
        Field<VEC> fc = cook<MODE, VEC, SCH, kG, PER>(A, rc0, act, edge_ok, edge_ok2);
        Field<VEC> um{}, uc_{};
        if constexpr (kR) {
            um = cook<MODE_RES, VEC, SCH, kG, PER>(A, as_res_row<MODE, VEC>(rm0), act && row_ok(y0 - 1),
                                                   edge_ok && row_ok(y0 - 1), edge_ok2 && row_ok(y0 - 1));
            uc_ = cook<MODE_RES, VEC, SCH, kG, PER>(A, as_res_row<MODE, VEC>(rc0), act, edge_ok, edge_ok2);
        }
        RawRow<MODE, VEC> rp = centre_row(y0 + 1);
        RawRow<MODE, VEC> ru{}, rd{};
        if (ld_u) ru = halo_row(y0, true);
        if (ld_d) rd = halo_row(y0, false);
        Row<VEC> unc{}, f0c{}, ax{};
        {
            const int64_t o = row_off(y0);
            if constexpr (kUn) unc = data_row<VEC, NK_ST_NTN>(A.un, o, true);
            if constexpr (kF0) f0c = data_row<VEC, NK_ST_NT>(A.F0, o, true);
            if constexpr (kAx) ax = data_row<VEC>(A.aux, o, true);
        }
        const int cnt = (int)(y1 - y0);
        for (int it = 0; it < cnt; ++it) {
            const int64_t j = y0 + it;
            const int64_t o = row_off(j);
            const int par = it & 1;
#pragma unroll
            for (int q = 0; q < VEC; ++q) {
                lz[par][0][wv][lane * VEC + q] = fc.c[q];
                if constexpr (kTG) lz[par][kTG ? 1 : 0][wv][lane * VEC + q] = fc.g[q];
                if constexpr (kR) lzu[par][kR ? wv : 0][kR ? lane * VEC + q : 0] = uc_.c[q];
            }
            // ---- issue: row j+2, the halo rows and centre data of row j+1
            const bool more = it + 1 < cnt;
            const int64_t j2 = more ? j + 2 : j + 1, j1 = more ? j + 1 : j;
            const RawRow<MODE, VEC> rpp = centre_row(j2);
            RawRow<MODE, VEC> ruu{}, rdd{};
            if (ld_u) ruu = halo_row(j1, true);
            if (ld_d) rdd = halo_row(j1, false);
            Row<VEC> uncn{}, f0cn{}, axn{};
            const int64_t o1 = row_off(j1);
            if constexpr (kUn) uncn = data_row<VEC, NK_ST_NTN>(A.un, o1, true);
            if constexpr (kF0) f0cn = data_row<VEC, NK_ST_NT>(A.F0, o1, true);
            if constexpr (kAx) axn = data_row<VEC>(A.aux, o1, true);
            // ---- cook what was issued one iteration ago
            const bool pok = row_ok(j + 1);
            const Field<VEC> fp = cook<MODE, VEC, SCH, kG, PER>(A, rp, act && pok, edge_ok && pok, edge_ok2 && pok);
            Field<VEC> fu{}, fd{};
            if (ld_u) fu = cook<MODE, VEC, SCH, kG, PER>(A, ru, act, false);
            if (ld_d) fd = cook<MODE, VEC, SCH, kG, PER>(A, rd, act, false);
            Field<VEC> up{}, fuu{}, fdu{};
            if constexpr (kR) {
                up = cook<MODE_RES, VEC, SCH, kG, PER>(A, as_res_row<MODE, VEC>(rp), act && pok, edge_ok && pok, edge_ok2 && pok);
                if (ld_u) fuu = cook<MODE_RES, VEC, SCH, kG, PER>(A, as_res_row<MODE, VEC>(ru), act, false);
                if (ld_d) fdu = cook<MODE_RES, VEC, SCH, kG, PER>(A, as_res_row<MODE, VEC>(rd), act, false);
            }
            __syncthreads();  // row j of every plane of the tile is in LDS
            double cu[VEC], cd[VEC], gu[VEC], gd[VEC];
#pragma unroll
            for (int q = 0; q < VEC; ++q) {
                cu[q] = lds_u ? lz[par][0][wv + (lds_u ? 1 : 0)][lane * VEC + q] : fu.c[q];
                cd[q] = lds_d ? lz[par][0][wv - (lds_d ? 1 : 0)][lane * VEC + q] : fd.c[q];
                if constexpr (kTG) {
                    gu[q] = lds_u ? lz[par][1][wv + (lds_u ? 1 : 0)][lane * VEC + q] : fu.g[q];
                    gd[q] = lds_d ? lz[par][1][wv - (lds_d ? 1 : 0)][lane * VEC + q] : fd.g[q];
                } else {
                    gu[q] = gd[q] = 0.0;
                }
            }
            double cuu[VEC], cdu[VEC];
            LR xu{};
            if constexpr (kR) {
#pragma unroll
                for (int q = 0; q < VEC; ++q) {
                    cuu[q] = lds_u ? lzu[par][kR ? wv + (lds_u ? 1 : 0) : 0][kR ? lane * VEC + q : 0] : fuu.c[q];
                    cdu[q] = lds_d ? lzu[par][kR ? wv - (lds_d ? 1 : 0) : 0][kR ? lane * VEC + q : 0] : fdu.c[q];
                }
                xu = x_nbrs<PER>(A, uc_.c[0], uc_.c[VEC - 1], uc_.e, uc_.e2, lane, xe.rwrap);
            }
            // ---- compute row j of my plane
            const LR xn = x_nbrs<PER>(A, fc.c[0], fc.c[VEC - 1], fc.e, fc.e2, lane, xe.rwrap);
            const double lft = xn.l, rgt = xn.r;
            double glft = 0.0, grgt = 0.0;
            if constexpr (SCH == 2 && kG) {
                const LR g2 = x_nbrs<PER>(A, fc.g[0], fc.g[VEC - 1], fc.ge, fc.ge2, lane, xe.rwrap);
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
                    const double lsum = (lapk(A, c, e, w, A.hx2, A.ihx2) + lapk(A, c, fp.c[q], fm.c[q], A.hy2, A.ihy2)) +
                                        lapk(A, c, cu[q], cd[q], A.hz2, A.ihz2);
                    double lsumg = 0.0;
                    if constexpr (SCH == 2 && kG) {
                        const double g = fc.g[q];
                        const double gw = (q == 0) ? glft : fc.g[q == 0 ? 0 : q - 1];
                        const double ge = (q == VEC - 1) ? grgt : fc.g[q == VEC - 1 ? q : q + 1];
                        lsumg = (lapk(A, g, ge, gw, A.hx2, A.ihx2) + lapk(A, g, fp.g[q], fm.g[q], A.hy2, A.ihy2)) +
                                lapk(A, g, gu[q], gd[q], A.hz2, A.ihz2);
                    }
                    const double unq = kG ? fc.g[q] : unc.v[q];
                    double f0 = f0c.v[q];
                    if constexpr (kR) {
                        const double uw = (q == 0) ? xu.l : uc_.c[q == 0 ? 0 : q - 1];
                        const double ue = (q == VEC - 1) ? xu.r : uc_.c[q == VEC - 1 ? q : q + 1];
                        const double ucc = uc_.c[q];
                        const double lsu = (lapk(A, ucc, ue, uw, A.hx2, A.ihx2) + lapk(A, ucc, up.c[q], um.c[q], A.hy2, A.ihy2)) +
                                           lapk(A, ucc, cuu[q], cdu[q], A.hz2, A.ihz2);
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
            ru = ruu;
            rd = rdd;
            unc = uncn;
            f0c = f0cn;
            ax = axn;
        }
    }
    if constexpr (EPI != EPI_NONE) publish<64 * NW>(acc, A.part, A.fin, sh, tz * A.tiles_x * A.tiles_y + txy);
}

// the variants' dispatch (nk_stencil.hpp's go_stencil, kernel-variant build): each returns what it launched
template <int KIND, int MODE, int EPI, int VEC, bool PER, int NW, bool F0R>
StInst go_st3y_i(const KArgs& A, int grid, hipStream_t s) {
    hipLaunchKernelGGL((k_st3y<KIND, MODE, EPI, VEC, PER, NW, F0R>), dim3(grid), dim3(64 * NW), 0, s, A);
    StInst r{};
    snprintf(r.name, sizeof r.name, "nk::k_st3y<%d, %d, %d, %d, %s, %d, %s>", KIND, MODE, EPI, VEC, st_tf(PER), NW,
             st_tf(F0R));
    r.f0r = F0R;
    return r;
}

template <int KIND, int MODE, int EPI, int NW>
StInst go_st3y(const KArgs& A, int vec, int grid, hipStream_t s, bool per) {
    constexpr bool kF0R = MODE == MODE_JFD && KIND == NK_HEAT3D_EULER;
    if constexpr (kF0R) {
        if (A.f0r) {
            if (per) return vec == 2 ? go_st3y_i<KIND, MODE, EPI, 2, true, NW, true>(A, grid, s)
                                     : go_st3y_i<KIND, MODE, EPI, 1, true, NW, true>(A, grid, s);
            return vec == 2 ? go_st3y_i<KIND, MODE, EPI, 2, false, NW, true>(A, grid, s)
                            : go_st3y_i<KIND, MODE, EPI, 1, false, NW, true>(A, grid, s);
        }
    }
    if (per) return vec == 2 ? go_st3y_i<KIND, MODE, EPI, 2, true, NW, false>(A, grid, s)
                             : go_st3y_i<KIND, MODE, EPI, 1, true, NW, false>(A, grid, s);
    return vec == 2 ? go_st3y_i<KIND, MODE, EPI, 2, false, NW, false>(A, grid, s)
                    : go_st3y_i<KIND, MODE, EPI, 1, false, NW, false>(A, grid, s);
}

template <int KIND, int MODE, int EPI, int VEC, bool PER, int NW>
StInst go_st3d_i(const KArgs& A, int grid, hipStream_t s) {
    hipLaunchKernelGGL((k_st3d<KIND, MODE, EPI, VEC, PER, NW>), dim3(grid), dim3(64 * NW), 0, s, A);
    StInst r{};
    snprintf(r.name, sizeof r.name, "nk::k_st3d<%d, %d, %d, %d, %s, %d>", KIND, MODE, EPI, VEC, st_tf(PER), NW);
    return r;
}

template <int KIND, int MODE, int EPI, int NW>
StInst go_st3d(const KArgs& A, int vec, int grid, hipStream_t s, bool per) {
    if (per) return vec == 2 ? go_st3d_i<KIND, MODE, EPI, 2, true, NW>(A, grid, s)
                             : go_st3d_i<KIND, MODE, EPI, 1, true, NW>(A, grid, s);
    return vec == 2 ? go_st3d_i<KIND, MODE, EPI, 2, false, NW>(A, grid, s)
                    : go_st3d_i<KIND, MODE, EPI, 1, false, NW>(A, grid, s);
}

template <int KIND, int MODE, int EPI, int VEC, bool PER, bool F0R, int NW>
StInst go_st2t_i(const KArgs& A, int grid, hipStream_t s) {
    hipLaunchKernelGGL((k_st2t<KIND, MODE, EPI, VEC, PER, F0R, NW>), dim3(grid), dim3(64 * NW), 0, s, A);
    StInst r{};
    snprintf(r.name, sizeof r.name, "nk::k_st2t<%d, %d, %d, %d, %s, %s, %d>", KIND, MODE, EPI, VEC, st_tf(PER),
             st_tf(F0R), NW);
    r.f0r = F0R;
    return r;
}

// one-shot LDS tiles: 8 rows x 128 columns (also 4 / 16 rows, and 256-column tiles for VEC 4)
template <int KIND, int MODE, int EPI>
StInst go_st2t(const KArgs& A, int vec, int grid, hipStream_t s, bool per) {
    if (vec == 4)  // 256 columns wide (no F0R / periodic)
        return A.tile2 == 4 ? go_st2t_i<KIND, MODE, EPI, 4, false, false, 4>(A, grid, s)
                            : go_st2t_i<KIND, MODE, EPI, 4, false, false, 8>(A, grid, s);
    auto go = [&](auto nwc) -> StInst {
        constexpr int NWc = decltype(nwc)::value;
        const bool f0r = MODE == MODE_JFD && A.f0r;
        if (per) {
            if constexpr (heat_kind<KIND>()) {
                return f0r ? go_st2t_i<KIND, MODE, EPI, 2, true, true, NWc>(A, grid, s)
                           : go_st2t_i<KIND, MODE, EPI, 2, true, false, NWc>(A, grid, s);
            }
        }
        return f0r ? go_st2t_i<KIND, MODE, EPI, 2, false, true, NWc>(A, grid, s)
                   : go_st2t_i<KIND, MODE, EPI, 2, false, false, NWc>(A, grid, s);
    };
    if (A.tile2 == 16) return go(std::integral_constant<int, 16>{});
    if (A.tile2 == 4) return go(std::integral_constant<int, 4>{});
    return go(std::integral_constant<int, 8>{});
}

}  // namespace
}  // namespace nk
