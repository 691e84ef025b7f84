// nk_halo.hip -- the distributed path's device side: the peer-mailbox binding and self-test, ghost
// planes of slabs (k_halo_ipc), the packed six-face exchange of 3D blocks (k_faces_ipc), the periodic
// wrap of a lone slab, and the policy helpers the stencil dispatch asks (in-launch ghost planes,
// self rings).  The reference's storage pattern is examples/halovector.jl:1-45 (ghost layer around
// the interior, filled by bc!); here the ghost layers are the neighbour ranks' boundary layers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "nk_device.hpp"

namespace nk {

// The binding (g_mb, one copy per translation unit and device) is process-wide: several contexts
// on one device share it.  A context binds its mailbox when it turns it on, and clears the binding
// only if it is the one bound -- tearing down a context without a mailbox (or another one's) must
// not unbind a live one.
namespace {
constexpr int kMaxDevices = 64;
nk_ctx* g_mb_owner[kMaxDevices] = {};
}  // namespace

int mailbox_bind(nk_ctx* c) {
    const int d = (c->device >= 0 && c->device < kMaxDevices) ? c->device : 0;
    if (!c->mb_on && g_mb_owner[d] != c) return NK_OK;
    g_mb_owner[d] = c->mb_on ? c : nullptr;
    MbInfo m{};
    if (c->mb_on) {
        m.self = c->mb_self;
        m.peers = c->mb_peers_dev;
        m.rank = c->rank;
        m.nranks = c->nranks;
        m.err = c->mb_err_dev;
        // polls before a mailbox wait gives up with an error (a few s: ranks may drift apart at start-up;
        // NK_MB_SPIN_LIMIT shortens it for the failure-path tests)
        const char* e = getenv("NK_MB_SPIN_LIMIT");
        m.spin_limit = (e && *e) ? (unsigned)atoll(e) : (1u << 26);
        if (!c->mb_wacc) {  // the peer-wait counters (nk_path_info), zeroed once per context
            NK_HIP(c, hipMalloc(reinterpret_cast<void**>(&c->mb_wacc), 4 * sizeof(unsigned long long)));
            NK_HIP(c, hipMemset(c->mb_wacc, 0, 4 * sizeof(unsigned long long)));
        }
        m.wacc = c->mb_wacc;
    }
    NK_HIP(c, hipMemcpyToSymbol(HIP_SYMBOL(g_mb), &m, sizeof(m)));
    // and the copy in every other unit: BLAS-1 / MGS, the stencil instantiations, the resident sweep
    for (auto bind : {kernels_bind_mb, stencil_bind_mb_1, stencil_bind_mb_2, stencil_bind_mb_3, stencil_bind_mb_4, stencil_bind_mb_5,
                      stencil_bind_mb_6, stencil_bind_mb_7, stencil_bind_mb_8, resident_bind_mb})
        NK_HIP(c, bind(m));
    return NK_OK;
}

namespace {
__global__ void k_mb_test(unsigned epoch, double value, double* out) {
    __shared__ double sh[kShN];
    mb_send(value, epoch);
    const double t = mb_recv(epoch, sh);
    if (threadIdx.x == 0) *out = t;
}
}  // namespace

namespace {

// Ghost planes through the peers' inboxes (IPC-mapped fine-grained memory over xGMI).  Block b
// owns chunk b of the plane: it pushes my boundary-plane chunks into the lower / upper
// neighbour's inbox (system-scope stores), drains, raises its epoch flag there, then waits for the
// neighbours' block b flags in my region and copies their chunks into my ghost planes.  Inboxes
// alternate by epoch parity: epoch e's push can only start after the neighbour finished epoch e-2.
// ring = 1 (bc_periodic! along the slab axis): rank 0's lower neighbour is rank nranks-1 and vice versa.
// Both sides' loads of an element round are issued before its stores (one memory latency per round).
__global__ __launch_bounds__(kBlock) void k_halo_ipc(double* __restrict__ v, int64_t plane, int64_t nplanes,
                                                    uint64_t epoch, int64_t cap, int ring) {
    __shared__ int ready;
    const int b = blockIdx.x, rank = g_mb.rank, nr = g_mb.nranks;
    const bool lo = rank > 0 || ring, hi = rank + 1 < nr || ring;
    const int rlo = rank > 0 ? rank - 1 : nr - 1, rhi = rank + 1 < nr ? rank + 1 : 0;
    const int par = (int)(epoch & 1);
    const int64_t per = (plane + gridDim.x - 1) / gridDim.x;
    const int64_t c0 = (int64_t)b * per, c1 = c0 + per < plane ? c0 + per : plane;
    const double* first = v;
    const double* last = v + (nplanes - 1) * plane;
    // my first interior plane -> the lower rank's "from upper" inbox, my last -> the upper rank's "from lower"
    uint64_t* dlo = lo ? halo_inbox(g_mb.peers[rlo], par, 1, cap) : nullptr;
    uint64_t* dhi = hi ? halo_inbox(g_mb.peers[rhi], par, 0, cap) : nullptr;
    for (int64_t i = c0 + threadIdx.x; i < c1; i += kBlock) {
        const double a = lo ? first[i] : 0.0, z = hi ? last[i] : 0.0;
        wait_loads();
        if (lo) __hip_atomic_store(dlo + i, (uint64_t)__double_as_longlong(a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (hi) __hip_atomic_store(dhi + i, (uint64_t)__double_as_longlong(z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every thread drains its stores before the flag
    __syncthreads();
    if (threadIdx.x < 64) {  // lane 0 the lower side, lane 1 the upper: flags raised and polled in parallel
        const int side = (int)threadIdx.x;
        const bool mine = (side == 0 && lo) || (side == 1 && hi);
        if (mine)
            __hip_atomic_store(halo_flags(g_mb.peers[side == 0 ? rlo : rhi]) + (par * kHaloSides + (side ^ 1)) * kHaloBlocks + b,
                               epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t t0 = wall_clock64();
        const bool ok = !mine || flag_wait(halo_flags(g_mb.self) + (par * kHaloSides + side) * kHaloBlocks + b, epoch);
        const bool all = __all(ok);
        if (side == 0) {
            ready = all ? 1 : 0;
            wait_note(kWaitHalo, t0);
        }
    }
    __syncthreads();
    if (!ready) return;
    const uint64_t* slo = halo_inbox(g_mb.self, par, 0, cap);
    const uint64_t* shi = halo_inbox(g_mb.self, par, 1, cap);
    for (int64_t i = c0 + threadIdx.x; i < c1; i += kBlock) {
        const uint64_t a = lo ? __hip_atomic_load(slo + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0;
        const uint64_t z = hi ? __hip_atomic_load(shi + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0;
        wait_loads();
        if (lo) v[i - plane] = __longlong_as_double((long long)a);
        if (hi) v[nplanes * plane + i] = __longlong_as_double((long long)z);
    }
}

// 3D blocks (nk_dist_grid): the six ghost layers of v through the peers' inboxes in ONE launch (packed
// faces).  Block b owns chunk b of every face: it pushes my boundary layer on each side s that has a
// neighbour into that neighbour's inbox for side s ^ 1 (system-scope stores), drains, raises its flag
// there, waits for the neighbours' block-b flags in my region and unpacks their layers -- the z ones into
// my ghost planes, the x / y ones into the faces after the allocation's trailing plane.  Neighbours share
// the face's extents, and the grid size is a constant, so both sides cut a face alike.  At a
// physical boundary the layer stays zero (zero-filled allocation, never written there).
struct FaceArgs {
    int64_t nx, ny, nz;
    int64_t fy, fx;  // offsets of the y-lo / x-lo faces from the interior pointer
    int nbr[kHaloSides];
};
__device__ __forceinline__ int64_t face_len(const FaceArgs& F, int s) {
    return s < 2 ? F.nx * F.ny : (s < 4 ? F.nx * F.nz : F.ny * F.nz);
}
// element i of my boundary layer on side s: planes (k fastest-y-x order of a plane), y faces k nx + x,
// x faces k ny + j
__device__ __forceinline__ int64_t face_src(const FaceArgs& F, int s, int64_t i) {
    const int64_t pl = F.nx * F.ny;
    if (s == 0) return i;
    if (s == 1) return (F.nz - 1) * pl + i;
    if (s < 4) return (i / F.nx) * pl + (s == 2 ? 0 : F.ny - 1) * F.nx + i % F.nx;
    return (i / F.ny) * pl + (i % F.ny) * F.nx + (s == 4 ? 0 : F.nx - 1);
}
// where element i of the layer from side s lands in my allocation
__device__ __forceinline__ int64_t face_dst(const FaceArgs& F, int s, int64_t i) {
    const int64_t pl = F.nx * F.ny;
    if (s == 0) return i - pl;
    if (s == 1) return F.nz * pl + i;
    if (s < 4) return F.fy + (s == 3 ? F.nx * F.nz : 0) + i;
    return F.fx + (s == 5 ? F.ny * F.nz : 0) + i;
}
__global__ __launch_bounds__(kBlock) void k_faces_ipc(double* __restrict__ v, FaceArgs F, uint64_t epoch, int64_t cap) {
    __shared__ int ready;
    const int b = blockIdx.x, G = gridDim.x;
    const int par = (int)(epoch & 1);
    // my chunk [c0, c1) of each face (empty where no neighbour); an element round issues the loads of all six
    // faces before any store -- one memory latency per round instead of one per face
    int64_t c0[kHaloSides], c1[kHaloSides], per_max = 0;
    uint64_t* dst[kHaloSides];
#pragma unroll
    for (int s = 0; s < kHaloSides; ++s) {
        const int64_t len = F.nbr[s] >= 0 ? face_len(F, s) : 0, per = (len + G - 1) / G;
        c0[s] = (int64_t)b * per;
        c1[s] = c0[s] + per < len ? c0[s] + per : len;
        per_max = per > per_max ? per : per_max;
        dst[s] = F.nbr[s] >= 0 ? halo_inbox(g_mb.peers[F.nbr[s]], par, s ^ 1, cap) : nullptr;
    }
    for (int64_t o = threadIdx.x; o < per_max; o += kBlock) {
        double val[kHaloSides];
#pragma unroll
        for (int s = 0; s < kHaloSides; ++s) val[s] = c0[s] + o < c1[s] ? v[face_src(F, s, c0[s] + o)] : 0.0;
        wait_loads();
#pragma unroll
        for (int s = 0; s < kHaloSides; ++s)
            if (c0[s] + o < c1[s])
                __hip_atomic_store(dst[s] + c0[s] + o, (uint64_t)__double_as_longlong(val[s]), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every thread drains its stores before the flags
    __syncthreads();
    if (threadIdx.x < 64) {  // lane s raises side s's flag and polls its own: six round trips in parallel
        const int s = (int)threadIdx.x;
        int nbr = -1;
#pragma unroll
        for (int q = 0; q < kHaloSides; ++q)
            if (q == s) nbr = F.nbr[q];
        if (nbr >= 0)
            __hip_atomic_store(halo_flags(g_mb.peers[nbr]) + (par * kHaloSides + (s ^ 1)) * kHaloBlocks + b, epoch,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t t0 = wall_clock64();
        const bool ok = nbr < 0 || flag_wait(halo_flags(g_mb.self) + (par * kHaloSides + s) * kHaloBlocks + b, epoch);
        const bool all = __all(ok);
        if (s == 0) {
            ready = all ? 1 : 0;
            wait_note(kWaitHalo, t0);
        }
    }
    __syncthreads();
    if (!ready) return;
    const uint64_t* src[kHaloSides];  // hoisted: the stores into v below could alias g_mb for the compiler
#pragma unroll
    for (int s = 0; s < kHaloSides; ++s) src[s] = halo_inbox(g_mb.self, par, s, cap);
    for (int64_t o = threadIdx.x; o < per_max; o += kBlock) {
        uint64_t val[kHaloSides];
#pragma unroll
        for (int s = 0; s < kHaloSides; ++s)
            val[s] = c0[s] + o < c1[s] ? __hip_atomic_load(src[s] + c0[s] + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0;
        wait_loads();
#pragma unroll
        for (int s = 0; s < kHaloSides; ++s)
            if (c0[s] + o < c1[s]) v[face_dst(F, s, c0[s] + o)] = __longlong_as_double((long long)val[s]);
    }
}

// bc_periodic! along the slab axis of a lone slab: ghost plane -1 <- the last interior plane,
// ghost plane nplanes <- the first (heat_2D.jl:20-21 / 23-24)
__global__ __launch_bounds__(kBlock) void k_periodic_fill(double* __restrict__ v, int64_t plane, int64_t nplanes) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < plane; i += (int64_t)gridDim.x * kBlock) {
        v[i - plane] = v[(nplanes - 1) * plane + i];
        v[nplanes * plane + i] = v[i];
    }
}
}  // namespace

int launch_halo_ipc(nk_ctx* c, double* v, int64_t plane, int64_t nplanes, bool ring) {
    if (halo_self_ring(c)) ring = true;
    else if (c->nranks < 2) return NK_OK;
    const uint64_t epoch = ++c->halo_epoch;
    static const int nb_env = std::max(1, std::min(kHaloBlocks, NK_TUNE("NK_HALO_NB", kHaloBlocks)));  // (kbench A/B)
    const int nb_max = std::min(nb_env, c->xchg_nb);
    int nb = (int)((plane + 1023) / 1024);
    if (nb > nb_max) nb = nb_max;
    if (nb < 1) nb = 1;
    const int nbrs = ring ? 2 : (c->rank > 0) + (c->rank + 1 < c->nranks);
    return launch(c, "halo_ipc", 16.0 * plane * nbrs, [&] {
        hipLaunchKernelGGL(k_halo_ipc, dim3(nb), dim3(kBlock), 0, c->stream, v, plane, nplanes, epoch, c->halo_cap,
                           ring ? 1 : 0);
    });
}

int launch_faces_ipc(nk_ctx* c, double* v, const nk_problem* p) {
    Geo g;
    NK_TRY(geometry(c, p, &g));
    FaceArgs F{};
    F.nx = p->nx;
    F.ny = p->ny;
    F.nz = p->nz;
    F.fy = g.n + g.plane;
    F.fx = F.fy + 2 * p->nx * p->nz;
    double bytes = 0.0;
    for (int s = 0; s < kHaloSides; ++s) {
        F.nbr[s] = block_nbr(c, s);
        if (F.nbr[s] >= 0) bytes += 16.0 * (double)(s < 2 ? p->nx * p->ny : (s < 4 ? p->nx * p->nz : p->ny * p->nz));
    }
    if (bytes == 0.0) return NK_OK;
    const uint64_t epoch = ++c->halo_epoch;
    // every rank cuts a face into the same nb chunks (xchg_nb is agreed at mailbox set-up, never the face's size)
    static const int nb_env = std::max(1, std::min(kHaloBlocks, NK_TUNE("NK_FACE_NB", kHaloBlocks)));  // (kbench A/B)
    const int nb = std::min(nb_env, c->xchg_nb);
    return launch(c, "halo_faces", bytes, [&] {
        hipLaunchKernelGGL(k_faces_ipc, dim3(nb), dim3(kBlock), 0, c->stream, v, F, epoch, c->halo_cap);
    });
}

int launch_periodic_fill(nk_ctx* c, double* v, int64_t plane, int64_t nplanes) {
    const int g = (int)std::min<int64_t>((plane + kBlock - 1) / kBlock, 1024);
    return launch(c, "periodic_fill", 16.0 * plane, [&] {
        hipLaunchKernelGGL(k_periodic_fill, dim3(g), dim3(kBlock), 0, c->stream, v, plane, nplanes);
    });
}

// every rank sends (rank + 1) (e + 1) for a few epochs; the sums must arrive exactly
int mailbox_selftest(nk_ctx* c, bool* ok) {
    *ok = true;
    for (int e = 0; e < 4; ++e) {
        const unsigned epoch = next_mb_epoch(c);
        hipLaunchKernelGGL(k_mb_test, dim3(1), dim3(64), 0, c->stream, epoch, (double)(c->rank + 1) * (e + 1), c->scal);
        NK_HIP(c, hipGetLastError());
        NK_HIP(c, hipMemcpyAsync(c->hpin, c->scal, sizeof(double), hipMemcpyDeviceToHost, c->stream));
        NK_HIP(c, hipStreamSynchronize(c->stream));
        const double want = (double)c->nranks * (c->nranks + 1) / 2 * (e + 1);
        if (c->hpin[0] != want || *c->mb_err) *ok = false;
    }
    return NK_OK;
}

// ghost planes / faces of a Krylov Jv inside the stencil launch when the peer mailbox is up (NK_HALO_FUSE=0, a
// rig like NK_HALO_SELF: the separate exchange kernels -- the same values, for A/B and the form tests)
int halo_fuse_knob() {
    static const int fuse = env_cfg("NK_HALO_FUSE", 1);
    return fuse;
}

// the points of the largest slab of an even split of the global grid along the slowest axis, from values
// every rank holds alike: the plane, the global spacing of that axis (h = 1 / (N + 1) with zero boundaries,
// the only ones whose ghost planes travel in the launch) and the rank count.  A spacing that names no grid
// gives the maximum: every rank then takes the exchange kernel.
int64_t shared_slab_points(const nk_ctx* c, const nk_problem* p, const Geo& g) {
    const double h = g.dim == 3 ? p->hz : g.dim == 2 ? p->hy : p->hx;
    if (!(h > 0.0) || !(1.0 / h < 1e15)) return INT64_MAX;
    const int64_t nglob = std::max<int64_t>(1, std::llround(1.0 / h) - 1);
    const int64_t nr = std::max(1, c->nranks);
    return g.plane * ((nglob + nr - 1) / nr);
}

// Measurement rigs (operational, like NK_RES_SHARED; they act only on a FORCED one-rank mailbox --
// NK_DIST_FORCE=1 NK_DIST_MAILBOX=1 -- which no solve of a real problem sets up):
// NK_HALO_SELF=1: the lone rank is its own lower and upper neighbour -- a self ring that runs the whole
// ghost-plane exchange on one GPU (tools/halo_self.py)
bool halo_self_ring(const nk_ctx* c) {
    static const int self = env_cfg("NK_HALO_SELF", 0);
    return self && c->mb_on && c->nranks == 1;
}
// NK_HALO_SELF=2: the lone rank is its own neighbour on all six sides of a 3D block -- the packed-face
// exchange and k_st3l's face reads of config 5's blocks on one GPU (bench.py --block-of, tools/halo_self.py)
bool block_self(const nk_ctx* c) {
    static const int self = env_cfg("NK_HALO_SELF", 0);
    return self == 2 && c->mb_on && c->nranks == 1;
}

}  // namespace nk
