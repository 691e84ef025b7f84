// nk_internal.hpp -- shared definitions of libnkhip.so (context, launch/profiling helpers,
// kernel-launcher prototypes).  Not part of the public ABI (that is include/nkhip.h).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <map>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "nkhip.h"

#include <rocprofiler-sdk-roctx/roctx.h>

namespace nk {

constexpr int kBlock = 256;          // threads per block for every streaming kernel (4 waves of 64)
constexpr int kMaxRedBlocks = 2048;  // partial sums per reduction (8 blocks per CU on 256 CUs)
constexpr int kRedSlots = 4;         // ring of partial-sum slots
constexpr int kRedCap = 16384;       // doubles per slot (a stencil launch may have more blocks)
constexpr int kTileCap = 1 << 19;    // one-shot stencil tiles per launch (per-tile partials before the group fold)
constexpr int kTileParts = 1024;     // partials a one-shot stencil launch hands on (tiles folded in groups)
constexpr int kScalCap = 8192;       // device scalar area (Hessenberg column, y, norms)
constexpr int kMaxUpdateVecs = 32;   // basis vectors folded per x-update launch
constexpr int kMgsVariant = 5;       // MGS-pass variant (unroll x non-temporal V_i), see mgs_dispatch

enum Mode { MODE_RES = 0, MODE_JEXACT = 1, MODE_JFD = 2 };
enum Epi {
    EPI_NONE = 0, EPI_SUMSQ = 1, EPI_DOT = 2, EPI_RESID = 3,
    EPI_DOTV = 4,   // kernel-internal: EPI_DOT + vout (V_k = v / h stored)
    EPI_DOTVS = 5   // kernel-internal: EPI_DOTV whose dot partner is that V_k itself (aux == nullptr)
};

struct ProfPending {
    int kid;
    hipEvent_t a, b;
    double bytes;
};
struct ProfAcc {
    int64_t launches = 0, timed = 0;
    double ms = 0.0, bytes = 0.0, bytes_all = 0.0, dram_all = 0.0;
    std::string kernel;  // the instantiation the class's last launch ran (stencils: StInst::name)
};

struct Comm;  // RCCL state (nk_dist.cpp)

}  // namespace nk

struct nk_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    std::unordered_map<double*, void*> allocs;  // interior pointer -> allocation base
    std::unordered_map<double*, int64_t> faced;  // 3D blocks: the vectors that carry x / y ghost faces (-> their size)
    unsigned alloc_seq = 0;                     // vectors allocated so far (their start offsets, §3)
    double* red = nullptr;                      // kRedSlots * kRedCap partial sums
    double* scal = nullptr;                     // kScalCap device scalars
    double* tpart = nullptr;                    // kTileCap per-tile partials of a one-shot stencil launch
    double* hpin = nullptr;                     // kScalCap pinned host scalars
    int red_next = 0;
    // profiling
    bool prof = false;
    int prof_every = 1;
    std::vector<nk::ProfPending> pending;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::string> kid_names;
    std::map<std::string, int> kid_of;
    std::vector<nk::ProfAcc> acc;
    // user kinds: the FD evaluation point w = u + eps v (one grid function, reallocated on a new geometry)
    double* user_w = nullptr;
    int64_t user_w_n = -1, user_w_plane = -1;
    // one-shot peer all-reduce of reduction scalars (nk_dist.cpp "mailbox"): fine-grained device
    // memory every rank can write over xGMI; epochs tag the granules
    bool mb_on = false;
    uint64_t* mb_self = nullptr;           // my mailbox (kMbSlots x kMbRanks x 2 granules)
    uint64_t** mb_peers_dev = nullptr;     // device table: rank -> that rank's mailbox (IPC-mapped)
    std::vector<void*> mb_opened;          // IPC mappings to close
    // host mailbox (NK_DIST_MAILBOX=host, or a peer's device invisible to this process): every rank's
    // region lives in a POSIX shared-memory segment, mapped and hipHostRegister-ed by every rank
    bool mb_host = false;                  // the active region (mb_self) is the host one
    uint64_t* mb_dev = nullptr;            // my device region (fine-grained device memory, IPC-shared)
    int64_t halo_cap_dev = 0;
    void* mb_host_base = nullptr;          // my host region: its mapping here,
    uint64_t* mb_host_dev = nullptr;       //   its device address,
    size_t mb_host_bytes = 0;
    int64_t halo_cap_host = 0;
    char mb_host_name[48] = {0};           //   its shared-memory name (unlinked once every peer mapped it)
    std::vector<std::pair<void*, size_t>> mb_host_maps;  // peers' segments mapped here
    int* mb_err = nullptr;                 // pinned host flag: a consumer timed out waiting for a peer
    unsigned long long* mb_wacc = nullptr; // device counters of the peer waits (nk_path_info): halo ticks, halo
                                           // waits, reduction ticks, reduction waits (device wall clock)
    int* mb_err_dev = nullptr;             // its device address
    unsigned mb_epoch = 1;
    int64_t halo_cap = 0;                  // doubles per inbox plane (0: no IPC halo exchange)
    uint64_t halo_epoch = 0;
    // resident MGS sweep (launch_mgs_sweep): one block per CU, q held in registers + LDS
    bool res_ok = true;                    // false when another rank shares this GPU (co-residency)
    // what actually ran (nk_dist_path): Krylov Jv launches whose v ghost planes travelled inside the
    // stencil launch / were exchanged by a separate launch first, resident sweeps, per-pass MGS launches
    int64_t n_jv_halo_fused = 0, n_jv_halo_separate = 0, n_sweep_resident = 0, n_mgs_pass = 0;
    // FD operator launches of the built-in stencils by instantiation: F(u) recomputed (F0R) / F0 loaded
    int64_t n_fd_f0r = 0, n_fd_f0_read = 0;
    uint64_t* res_gran = nullptr;          // partial-sum granules: 2 parities x res_blocks x 2
    int* res_err = nullptr;                // pinned host flag: a granule poll timed out
    int* res_err_dev = nullptr;
    unsigned res_tag = 0;                  // granule tags handed out so far
    int res_blocks = 0, res_rl = 0;        // grid (= CUs) and LDS double2 slots per thread
    int res_share = 1;                     // ranks on this GPU (NK_RES_SHARED: each sweep grid gets CUs / res_share)
    int share_most = 1;                    // the most ranks on any one GPU -- the same on every rank (mailbox set-up)
    int n_cus = 0;                         // the device's CU count (0: not queried yet)
    int* blk_order = nullptr;              // 3D blocks, in-launch exchange: the tile dispatch order (device), its
    int blk_order_cap = 0;                 //   capacity and the geometry it was built for
    uint64_t blk_order_key = 0;
    int xchg_nb = 256;                     // exchange-kernel grid (<= kHaloBlocks), the same on every rank: kHaloBlocks / the most
                                           // ranks sharing one GPU, so every sharing rank's spinning exchange grid fits at once
    uint64_t* res_tstamp = nullptr;        // kernel-variant bench only (nkb_mgs_res, NK_RES_TSTAMP)
    // pipelined ILU(0) sweeps (launch_ilu0_*): per-strip progress counters + a pinned timeout flag
    int64_t* ilu_prog = nullptr;
    int64_t ilu_prog_cap = 0;
    int* ilu_err = nullptr;
    bool ilu_redo = false;                 // a pipelined ILU(0) sweep timed out: the caller redoes its work (level sweep)
    int* ilu_err_dev = nullptr;
    bool ilu_pipe_ok = true;               // false after a progress poll timed out: the one-work-group sweep
    // distribution: nranks = px * py * pz ranks; px = py = 1 (the default) is the slab decomposition along the
    // slowest axis, otherwise 3D problems are split into blocks (rank = (iz py + iy) px + ix, nk_dist_grid)
    int rank = 0, nranks = 1;
    int px = 1, py = 1;
    nk::Comm* comm = nullptr;
};

namespace nk {

// Operational configuration from the environment (unset or empty: dflt): the transport of the
// distributed path, timeouts, shared-GPU test rigs.  None of them changes a kernel's arithmetic;
// DESIGN.md §5 lists them.
inline int env_cfg(const char* name, int dflt) {
    const char* s = getenv(name);
    return (s && *s) ? atoi(s) : dflt;
}
// Kernel-variant tuning knobs (tile shapes, grid sizes, load flavours, experimental variants): read
// from the environment only in the kernel-variant bench build (lib/libnkhip_kbench.so, -DNK_KBENCH,
// driven by tools/); the product library compiles the default in and reads nothing.
#ifdef NK_KBENCH
#define NK_TUNE(name, dflt) ::nk::env_cfg(name, dflt)
#else
#define NK_TUNE(name, dflt) (dflt)
#endif

// ---------------------------------------------------------------- errors
int fail(nk_ctx* c, int code, const std::string& msg);
#define NK_HIP(c, expr)                                                                         \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return ::nk::fail((c), NK_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)
#define NK_TRY(expr)             \
    do {                         \
        int r_ = (expr);         \
        if (r_ != NK_OK) return r_; \
    } while (0)

// ---------------------------------------------------------------- grid geometry
struct Geo {
    int dim;          // 1, 2, 3
    int64_t n;        // interior points
    int64_t plane;    // ghost-plane size along the slowest axis (1, nx, nx*ny)
    int64_t nplanes;  // interior planes along the slowest axis
    int64_t front;    // doubles before the interior (>= plane, multiple of 32 => 256-B aligned interior)
};
int geometry(nk_ctx* c, const nk_problem* p, Geo* g);

// ---------------------------------------------------------------- profiling helpers
int kid(nk_ctx* c, const char* name);
int prof_begin(nk_ctx* c, hipEvent_t* a);
int prof_end(nk_ctx* c, int k, hipEvent_t a, double bytes);
void prof_drain(nk_ctx* c, bool blocking);

// run `f()` (which enqueues one kernel on c->stream and returns that launch's algorithmic operand bytes
// -- every load / store it must issue, served by any cache level -- for the instantiation it actually
// dispatched) under optional event timing.  dram: the unique-DRAM model of the same launch (each
// distinct operand byte once; < 0: = bytes); kernel (optional): the instantiation's name for the profile
template <typename F>
int launch_dyn(nk_ctx* c, const char* name, F&& f, double dram = -1.0, const char* const* kernel = nullptr) {
    hipEvent_t a = nullptr;
    int k = -1;
    bool timed = false;
    if (c->prof) {
        k = kid(c, name);
        timed = (c->acc[k].launches++ % c->prof_every) == 0;
        if (timed) NK_TRY(prof_begin(c, &a));
    }
    const double bytes = f();
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(c, NK_E_HIP, std::string("launch ") + name + ": " + hipGetErrorString(e));
    if (c->prof) {
        c->acc[k].bytes_all += bytes;
        c->acc[k].dram_all += dram < 0.0 ? bytes : dram;
        if (kernel && *kernel) c->acc[k].kernel = *kernel;
    }
    if (timed) NK_TRY(prof_end(c, k, a, bytes));
    return NK_OK;
}
// the same for a kernel whose bytes do not depend on the dispatch
template <typename F>
int launch(nk_ctx* c, const char* name, double bytes, F&& f, double dram = -1.0) {
    return launch_dyn(c, name, [&] { f(); return bytes; }, dram);
}

// ---------------------------------------------------------------- reductions
// A reduction result lives either as `len` partial sums (single rank) or, after finish_reduction
// on several ranks, as one all-reduced scalar.  Consumers sum `len` doubles at `ptr` in a fixed
// order, so every block (and every run) sees the bit-identical value.
struct Red {
    const double* ptr;
    int len;                // < 0: -(1 + (epoch << 15 | count)): cross-rank through the peer mailbox
    double* fin = nullptr;  // multi-rank: the producing kernel already folded its partials here
    unsigned epoch = 0;     // mailbox epoch the producing kernel published under (0: none)
};
double* red_slot(nk_ctx* c);                 // next partial-sum slot of the ring
unsigned next_mb_epoch(nk_ctx* c);           // the next peer-mailbox epoch (1 .. 65535)
double* red_out(nk_ctx* c, int len, Red* r, int* fin);  // slot for a reduction launch (+ fold flag)
int finish_reduction(nk_ctx* c, Red* r);     // multi-rank: collapse + RCCL all-reduce
int mb_check(nk_ctx* c);                     // after a host sync: did a mailbox wait time out?
int red_blocks(int64_t n);                   // grid size of streaming reductions
bool halo_self_ring(const nk_ctx* c);        // rig (NK_HALO_SELF=1): a forced one-rank mailbox exchanges ghost planes with itself
int halo_fuse_knob();                        // 1: a Krylov Jv's ghost planes travel in the stencil launch (mailbox up)
// One Arnoldi step's MGS sweep in one launch (np passes over V[t % k], then ||q||) with q resident
// on chip; returns 1 (nothing enqueued) when the resident path does not apply.
// *vout (optional): where to store V_{k+1} = q / ||q|| instead of q; reset to null when the sweep
// stores q (not every slot resident).
// *jin (optional, 2D Bratu FD Jv at full residency only): compute q = J V_k in the launch itself
// (q never touches memory; `in` is unused) -- returns 1 without enqueueing when it does not apply.
struct ResJv {
    const double *u, *v, *F0, *aux;  // u, V_k, F(u), V_1
    double eps, lam, hx2, hy2;
    int64_t nx;
};
int launch_mgs_sweep(nk_ctx* c, int64_t n, double* q, const double* const* V, int k, int np, Red in, double* col,
                     double* colh, int rv, double** vout, const ResJv* jin = nullptr);
constexpr int kMbSlots = 256;                // mailbox ring (epoch % kMbSlots)
constexpr int kMbRanks = 32;                 // max ranks of the mailbox all-reduce (2 granules each: one wave polls them all)
constexpr int kHaloBlocks = 256;              // blocks (= flags per side) of the IPC ghost-plane exchange
constexpr int kHaloSides = 6;                // ghost layers by the side they come from: 0 / 1 the slowest axis's lower /
                                             // upper neighbour (slabs; z of 3D blocks), 2 / 3 y, 4 / 5 x (3D blocks)
constexpr int kHaloTileFlags = 4096;         // stencil tiles per plane whose ghost patch travels in the stencil itself
constexpr int64_t kSharedFuseMax = (int64_t)1 << 20;  // ranks sharing a GPU: in-launch ghost planes up to this many points
// per slab (rank-uniform estimate: shared_slab_points); NK_SHARED_FUSE_MAX overrides it (test rigs)
int64_t shared_slab_points(const nk_ctx* c, const nk_problem* p, const Geo& g);
// one fine-grained region per rank, IPC-mapped by every other rank:
//   [mailbox: kMbSlots x kMbRanks x 2 u64][halo flags: 2 parity x kHaloSides x kHaloBlocks u64]
//   [tile flags: 2 parity x kHaloSides sides x kHaloTileFlags u64]  (slab ends: sides 0 / 1; 3D blocks: all six)
//   [halo inbox: 2 parity x kHaloSides x halo_cap doubles]   (side 0: from the lower rank, 1: from the upper, ...)
constexpr size_t kMbWords = (size_t)2 * kMbSlots * kMbRanks;
constexpr size_t kHaloFlagWords = (size_t)2 * kHaloSides * kHaloBlocks + (size_t)2 * kHaloSides * kHaloTileFlags;
int mailbox_bind(nk_ctx* c);                 // make c's mailbox the one the kernels use (nk_kernels.hip)
int mailbox_selftest(nk_ctx* c, bool* ok);   // a few epochs through the mailbox vs the expected sums
// ghost planes of v (interior pointer, `plane` doubles per plane, `nplanes` planes) through the peer
// inboxes: push my boundary planes into the neighbours' inboxes, pull theirs into my ghost planes
int launch_halo_ipc(nk_ctx* c, double* v, int64_t plane, int64_t nplanes, bool ring);
// 3D blocks: the six ghost layers of v (z planes in the allocation, x / y faces after it) through the inboxes
int launch_faces_ipc(nk_ctx* c, double* v, const nk_problem* p);
int launch_periodic_fill(nk_ctx* c, double* v, int64_t plane, int64_t nplanes);

// ---------------------------------------------------------------- kernel launchers (nk_kernels.hip)
struct StencilIn {
    const nk_problem* p;
    int mode;          // Mode
    int epi;           // Epi
    double* out;
    const double* u;
    const double* v;
    const double* F0;
    const double* aux; // EPI_DOT: dot partner; EPI_RESID: b (out = b - J v)
    double eps;
    const double* vdiv = nullptr;  // device scalar h: the operator is applied to v / h ...
    double* vout = nullptr;        // ... and v / h is stored here (fused kdivcopy!)
    bool xchg_v = false;           // v's ghost planes are stale: exchange them (in the stencil itself when
                                   // the peer mailbox is up, else halo_exchange before the launch)
    bool f0r = false;              // FD: F0 is exactly F(u) as this library's residual kernel computed it, so
                                   // the 2D kernels recompute it in registers instead of loading it
};
// returns the partial sums (when epi != EPI_NONE) in *red
int launch_stencil(nk_ctx* c, const StencilIn& in, Red* red);
// the same with the kernel-variant bench's overrides (rows / planes per tile, variant bits; 0, 0: the product)
int launch_stencil_ex(nk_ctx* c, const StencilIn& in, Red* red, int rows_override, int fast);
int wide_blocks(int64_t n);                  // grid of the streaming kernels whose partials only a finaliser reads

int launch_dot(nk_ctx* c, int64_t n, const double* x, const double* y, Red* red);
int launch_sumsq(nk_ctx* c, int64_t n, const double* x, Red* red);
int launch_finalize(nk_ctx* c, Red r, double* dst, int sqrt_it, double* mirror = nullptr);  // dst[0] = sum (or sqrt(sum))
int launch_axpy(nk_ctx* c, int64_t n, double s, const double* x, double* y);
int launch_axpy_sumsq(nk_ctx* c, int64_t n, double s, const double* x, double* y, Red* red);  // + ||y||^2 partials
int launch_axpby(nk_ctx* c, int64_t n, double s, const double* x, double t, double* y);
int launch_scal(nk_ctx* c, int64_t n, double s, double* x);
int launch_copy(nk_ctx* c, int64_t n, double* y, const double* x);
int launch_fill(nk_ctx* c, int64_t n, double* x, double v);
int launch_divcopy(nk_ctx* c, int64_t n, double* y, const double* x, double s);
int launch_ref(nk_ctx* c, int64_t n, double* x, double* y, double cc, double ss);
int launch_exp(nk_ctx* c, int64_t n, double* y, const double* x);
// one fused modified-Gram-Schmidt pass: h = Σ in; q -= h vi; partials of <vnext, q> (or <q,q>
// when vnext == nullptr).  Block 0 stores h at h_out (and at h_host, a mapped host address, if given).
int launch_mgs_pass(nk_ctx* c, int64_t n, double* q, const double* vi, const double* vnext, Red in,
                    double* h_out, double* h_host, Red* out, int rev);
// xr = Σ_i y_i V_i (fma chain from 0 in i order, y on device); then x = x + xr (restart) or
// x = xr; optional partial sums of ||x||^2.
// u (optional): the Newton update is fused into the last chunk -- u -= x_final, x is NOT stored,
// and xnorm receives ||u||^2 partials instead of ||x||^2.
int launch_update_x(nk_ctx* c, int64_t n, double* x, double* xr, const double* const* V, int k,
                    const double* y_dev, int restart, Red* xnorm, double* u = nullptr);
// CG pieces: x += a p ; r -= a Ap ; partial <r,r>   and   p = r + b p
int launch_cg_update(nk_ctx* c, int64_t n, double alpha, double* x, double* r, const double* p,
                     const double* Ap, Red* rr);
int launch_cg_direction(nk_ctx* c, int64_t n, double beta, double* p, const double* r);
int launch_diag_apply(nk_ctx* c, int64_t n, double* z, const double* d, const double* v, Red* red);  // z = d .* v (+ ||z||^2)
int launch_jdiag(nk_ctx* c, const nk_problem* p, double* out, const double* u, int recip);        // diag(J(u)) or 1 ./ diag
int launch_ilu0_factor(nk_ctx* c, const nk_problem* p, int dim, double* d);                       // diag(J) -> D~ (in place)
int launch_ilu0_solve(nk_ctx* c, const nk_problem* p, int dim, const double* d, double* z, const double* v);  // z = (LU)^-1 v
// after a pipelined ILU(0) launch: 1 if its progress poll timed out (output partial; the pipelined path
// is now off for this context), 0 if it completed, < 0 on a HIP error
int ilu_pipe_failed(nk_ctx* c);
// NK_USER pieces: w = u + eps (v / *vdiv) (w may be null) and vout = v / *vdiv (vout may be null);
// and the epilogue pass after a user F / J: out = (out - F0) / eps when fd, + the `epi` partials.
int launch_fd_point(nk_ctx* c, int64_t n, double* w, const double* u, const double* v, const double* vdiv,
                    double eps, double* vout);
int launch_user_epi(nk_ctx* c, int64_t n, int fd, double* out, const double* F0, double eps, int epi,
                    const double* aux, Red* red);
int launch_user(nk_ctx* c, const StencilIn& in, Red* red);  // nk_user.cpp
// roctx range for the lifetime of a scope (shows Newton steps / Krylov solves / GMRES cycles in
// rocprofv3 --marker-trace timelines; a no-op when no profiler is attached)
struct Range {
    explicit Range(const char* name) { roctxRangePush(name); }
    ~Range() { roctxRangePop(); }
    Range(const Range&) = delete;
    Range& operator=(const Range&) = delete;
};

inline bool nk_is_user(int kind) { return kind >= NK_USER1D && kind <= NK_USER3D; }
inline bool nk_is_heat(int kind) { return kind >= NK_HEAT2D_EULER && kind <= NK_HEAT3D_TRAPEZOID; }
// implicit.jl scheme of a heat kind: 0 G_Euler!, 1 G_Midpoint!, 2 G_Trapezoid!
inline int nk_scheme(int kind) {
    return (kind == NK_HEAT2D_MIDPOINT || kind == NK_HEAT3D_MIDPOINT) ? 1
           : ((kind == NK_HEAT2D_TRAPEZOID || kind == NK_HEAT3D_TRAPEZOID) ? 2 : 0);
}

// ---------------------------------------------------------------- distribution (nk_dist.cpp)
// 3D blocks (nk_dist_grid with px * py > 1): a 3D grid function's allocation carries, after its trailing
// z ghost plane, the four x / y ghost faces the neighbours' boundary layers are exchanged into:
//   [y-lo: nx nz][y-hi: nx nz][x-lo: ny nz][x-hi: ny nz]   (y faces indexed k nx + i, x faces k ny + j)
bool block_self(const nk_ctx* c);  // rig (NK_HALO_SELF=2): a forced one-rank mailbox is its own neighbour on all six sides
inline bool blocks3d(const nk_ctx* c, const Geo& g) { return g.dim == 3 && (c->px * c->py > 1 || block_self(c)); }
inline int64_t face_words(const nk_ctx* c, const nk_problem* p, const Geo& g) {
    return blocks3d(c, g) ? 2 * (p->nx + p->ny) * p->nz : 0;
}
// the neighbour rank on side s (kHaloSides numbering) of a 3D block, -1 at a physical boundary
int block_nbr(const nk_ctx* c, int side);
int halo_exchange(nk_ctx* c, const nk_problem* p, const double* v);
// ghost planes of u_n when the residual reads its neighbours (G_Midpoint!, G_Trapezoid!)
int exchange_un(nk_ctx* c, const nk_problem* p);
int allreduce_scalar(nk_ctx* c, double* dev, int64_t count);

}  // namespace nk
