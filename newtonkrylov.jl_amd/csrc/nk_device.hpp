// nk_device.hpp -- device-side primitives shared by the kernel translation units: fixed-order
// block reductions, the peer-mailbox all-reduce (mb_send / mb_recv), the partial-sum hand-off
// (publish).  Included by nk_kernels.hip and by every stencil instantiation unit
// (nk_stencil_inst.hip); everything here has internal linkage, so each unit owns its own copy of
// the g_mb binding, which mailbox_bind (nk_kernels.hip) sets in every unit.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#include "nk_internal.hpp"

#include "nk_exp_dev.hpp"

namespace nk {

// mailbox binding of one rank (set by mailbox_bind)
struct MbInfo {
    uint64_t* self;
    uint64_t* const* peers;
    int rank, nranks;
    int* err;            // pinned host flag
    unsigned spin_limit;
    unsigned long long* wacc;  // peer-wait accounting (nk_path_info): [2w] ticks, [2w + 1] waits; w = 0 ghost
                               // planes, 1 cross-rank reductions (null: not counted)
};
hipError_t resident_bind_mb(const MbInfo& m);  // nk_resident.hip's copy of g_mb
hipError_t kernels_bind_mb(const MbInfo& m);   // nk_kernels.hip's copy
// the stencil instantiation units' copies (nk_stencil_inst.hip, one per problem kind)
hipError_t stencil_bind_mb_1(const MbInfo& m);
hipError_t stencil_bind_mb_2(const MbInfo& m);
hipError_t stencil_bind_mb_3(const MbInfo& m);
hipError_t stencil_bind_mb_4(const MbInfo& m);
hipError_t stencil_bind_mb_5(const MbInfo& m);
hipError_t stencil_bind_mb_6(const MbInfo& m);
hipError_t stencil_bind_mb_7(const MbInfo& m);
hipError_t stencil_bind_mb_8(const MbInfo& m);

typedef double dx2 __attribute__((ext_vector_type(2)));  // 16-B streaming element

namespace {

// ------------------------------------------------------------------------------ streaming order
// Block-contiguous chunks of `len` elements (a multiple of the block size), threads interleaved
// inside the chunk: each block streams one address range -- fewer DRAM page switches than the
// grid-stride order once the vectors outgrow the Infinity Cache (tools/stream_probe.py).
struct Chunk {
    int64_t lo, hi;
};
__device__ __forceinline__ Chunk block_chunk(int64_t len) {
    const int64_t per = ((len + gridDim.x - 1) / gridDim.x + kBlock - 1) / kBlock * kBlock;
    const int64_t lo = (int64_t)blockIdx.x * per;
    return Chunk{lo, lo + per < len ? lo + per : len};
}
#define NK_CHUNKED(i, len)                    \
    const Chunk ck_ = block_chunk(len);       \
    for (int64_t i = ck_.lo + threadIdx.x; i < ck_.hi; i += kBlock)

// 16-B loads / stores, non-temporal (NT: streamed past the caches' retention) or plain
template <bool NT>
__device__ __forceinline__ dx2 ld2(const dx2* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NT>
__device__ __forceinline__ void st2(dx2* p, dx2 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// ------------------------------------------------------------------------------ reductions
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;  // lane 0's value is used: a fixed association order
}

// sum over the NT threads of the block (NT / 64 waves, at most 16); valid in thread 0.  The wave sums
// go to sh[0 .. NT/64) and are added in wave order (((w0 + w1) + w2) + ...); sh[kShB] is the slot
// the callers broadcast through, disjoint from every wave slot.
constexpr int kShB = 16, kShN = 17;
template <int NT = kBlock>
__device__ __forceinline__ double block_sum(double v, double* sh) {
    static_assert(NT % 64 == 0 && NT / 64 <= kShB, "block_sum: 1 .. 16 waves");
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    double r = 0.0;
    if (threadIdx.x == 0) {
        r = sh[0];
#pragma unroll
        for (int k = 1; k < NT / 64; ++k) r += sh[k];
    }
    return r;
}

// fixed-order sum of in[0..len), broadcast to the whole block.  All 256 threads load (8
// independent loads in flight each), so a block pays ~one L2 round trip, not 32 dependent ones.
// ------------------------------------------------------------------------------ peer mailbox
// One-shot all-reduce of a reduction scalar across ranks without a collective launch: the
// producing kernel's last block writes its folded value into EVERY rank's mailbox (fine-grained
// device memory, IPC-mapped over xGMI), the consuming kernel polls the nranks entries of its own
// mailbox and sums them in rank order -- the same order on every rank, so every rank holds the
// bit-identical scalar.  Each 64-bit value travels as two self-validating 8-byte granules
// {epoch:32 | half:32} (cdna_hip_programming.md §6 G16, R2: no flag, no fence, no tearing).
// Spins are bounded: a peer that never arrives sets the error flag instead of hanging the GPU.
// one copy of g_mb per translation unit (internal linkage): mailbox_bind sets every copy
__device__ MbInfo g_mb;

// one peer wait's device wall-clock time (ticks since t0) into the context's counters
constexpr int kWaitHalo = 0, kWaitReduce = 1;
__device__ __forceinline__ void wait_note(int which, uint64_t t0) {
    if (!g_mb.wacc) return;
    const unsigned long long dt = (unsigned long long)(wall_clock64() - t0);
    __hip_atomic_fetch_add(g_mb.wacc + 2 * which, dt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(g_mb.wacc + 2 * which + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t* mb_cell(uint64_t* base, unsigned epoch, int rank) {
    return base + ((size_t)(epoch % kMbSlots) * kMbRanks + rank) * 2;
}

// lanes r < nranks (first wave) send {epoch, t} to rank r
__device__ __forceinline__ void mb_send(double t, unsigned epoch) {
    const int l = threadIdx.x;
    if (l < g_mb.nranks) {
        const uint64_t bits = (uint64_t)__double_as_longlong(t);
        const uint64_t tag = (uint64_t)epoch << 32;
        uint64_t* cell = mb_cell(g_mb.peers[l], epoch, g_mb.rank);
        __hip_atomic_store(cell, tag | (bits & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(cell + 1, tag | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Σ_r value_r of `epoch` in rank order, broadcast to the whole block (all threads must call)
__device__ double mb_recv(unsigned epoch, double* sh) {
    if (threadIdx.x < 64) {
        const int l = threadIdx.x, nr = g_mb.nranks;
        const uint64_t t0 = (blockIdx.x == 0 && l == 0) ? wall_clock64() : 0;
        uint32_t half = 0;
        if (l < 2 * nr) {
            const uint64_t* g = mb_cell(g_mb.self, epoch, l >> 1) + (l & 1);
            uint64_t x = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            unsigned spins = 0;
            while ((unsigned)(x >> 32) != epoch) {
                // bounded: past spin_limit polls raise the error flag; and once ANY wait of this rank
                // has timed out (a dead peer), every later one gives up within 256 polls -- so a failed
                // rank costs its peers one timeout per host sync, not one per consuming kernel
                if (++spins > g_mb.spin_limit ||
                    ((spins & 255) == 0 && __hip_atomic_load(g_mb.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))) {
                    __hip_atomic_store(g_mb.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    x = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
                x = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            half = (uint32_t)x;
        }
        const uint32_t hi = __shfl_down(half, 1, 64);
        const double v = __longlong_as_double((long long)(((uint64_t)hi << 32) | half));
        double t = 0.0;
        for (int r = 0; r < nr; ++r) t += __shfl(v, 2 * r, 64);  // fixed rank order
        if (l == 0) sh[kShB] = t;
        if (blockIdx.x == 0 && l == 0) wait_note(kWaitReduce, t0);  // (every lane's poll has ended here)
    }
    __syncthreads();
    return sh[kShB];
}

// SC1 = true reads with agent-scope (sc1) loads: values other blocks of the SAME launch stored
// write-through (publish), which this CU's L1 or this XCD's L2 may hold stale copies of.
template <bool SC1 = false>
__device__ __forceinline__ double ld_part(const double* p) {
    if constexpr (SC1) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return *p;
}

// A reduction handed to a consumer kernel: `len` partial sums at `in`, summed in a fixed order.
// len < 0 encodes a cross-rank reduction through the peer mailbox: -(1 + (epoch << 15 | count)).
// Every block sums this rank's `count` partials (the same value in every block), block 0 sends it
// to every rank's mailbox under `epoch`, and all blocks wait for the nranks values and add them in
// rank order -- no arrival ticket or serial fold at the end of the producing kernel.  (Block 0 is
// dispatched first, so the blocks that wait cannot starve the sender.)
__device__ __forceinline__ int mb_encode(unsigned epoch, int count) { return -(1 + (int)((epoch << 15) | (unsigned)count)); }

template <bool SC1 = false, int NT = kBlock>
__device__ __forceinline__ double reduce_input(const double* __restrict__ in, int len, double* sh) {
    unsigned epoch = 0;
    if (len < 0) {
        const unsigned code = (unsigned)(-len - 1);
        epoch = code >> 15;
        len = (int)(code & 0x7fffu);
    }
    double t = 0.0;
    int m = threadIdx.x;
    for (; m + 7 * NT < len; m += 8 * NT) {
        double a[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) a[r] = ld_part<SC1>(in + m + r * NT);
#pragma unroll
        for (int r = 0; r < 8; ++r) t += a[r];
    }
    for (; m < len; m += NT) t += ld_part<SC1>(in + m);
    t = block_sum<NT>(t, sh);
    if (threadIdx.x == 0) sh[kShB] = t;
    __syncthreads();
    if (epoch == 0) return sh[kShB];
    const double mine = sh[kShB];
    if (blockIdx.x == 0) mb_send(mine, epoch);
    __syncthreads();  // every thread has read sh[kShB] before mb_recv reuses it
    return mb_recv(epoch, sh);
}

// Block partial -> part[blockIdx.x].  With `fin` (a communicator is attached) the last block to
// arrive also folds all partials -- the same fixed-order sum k_finalize computes -- into
// part[kRedCap - 1], so the RCCL all-reduce can follow without a separate finaliser launch.  The
// arrival counter lives in part[kRedCap - 2] and is reset by that last block.
// Hand-off without fences (cdna_hip_programming.md §6 Guideline 16, R1/R2 forms): the partial is
// stored write-through (agent-scope atomic store = sc1) and drained before the ticket; the last
// block reads the partials with sc1 loads.  An agent-scope RELEASE fence here would write back the
// XCD's whole L2 -- full of this kernel's streamed output -- once per block (measured: 2x slower).
// slot: where the partial goes (default: blockIdx.x).  The stencils pass their TILE index, so the
// fixed-order sum runs over tiles in address order whatever block a tile was dispatched on (the XCD
// bands, the slab-end tiles first when ghost planes travel in the launch): the same operator gives the
// same bits on every path.
// publish_sum: the same for a value already reduced (valid in thread 0), one of n partials
template <int NT = kBlock>
__device__ __forceinline__ void publish_sum(double s, double* part, int fin, double* sh, int slot, int n) {
    __shared__ unsigned ticket;
    if (!fin) {
        if (threadIdx.x == 0) part[slot] = s;
        return;
    }
    unsigned* cnt = reinterpret_cast<unsigned*>(part + kRedCap - 2);
    if (threadIdx.x == 0) {  // the partial's only writer is this lane
        __hip_atomic_store(part + slot, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ticket = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (ticket != (unsigned)(n - 1)) return;
    const double t = reduce_input<true, NT>(part, n, sh);
    if (threadIdx.x == 0) {
        part[kRedCap - 1] = t;
        __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (fin >= 2) mb_send(t, (unsigned)fin);  // fin = mailbox epoch: straight to every rank
}
template <int NT = kBlock>
__device__ __forceinline__ void publish(double acc, double* part, int fin, double* sh, int slot = -1) {
    const double s = block_sum<NT>(acc, sh);
    publish_sum<NT>(s, part, fin, sh, slot < 0 ? (int)blockIdx.x : slot, (int)gridDim.x);
}
__device__ __forceinline__ double lap(double c, double p, double m, double h2) { return ((p - 2.0 * c) + m) / h2; }

// ------------------------------------------------------------------------------ peer ghost planes
// One wait for a batch of loads (vmcnt(0) lgkmcnt(0), gfx9 encoding).  The exchanges load a round of
// elements, wait once, then store them all: a load issued after a system-scope store can only be waited
// for together with that store's acknowledgement (one in-order vmcnt), so a load -> store loop pays one
// store round trip per element -- over fine-grained memory about a microsecond each.  (Without the explicit
// wait the waitcnt pass also loses the count at the predicated stores' join points and waits before each.)
__device__ __forceinline__ void wait_loads() { __builtin_amdgcn_s_waitcnt(0x0070); }
// elements per thread per exchange round: a 2D slab tile's patch (one 512-column row) is 2 per thread; a 3D
// block tile's y patch 8 (two rounds).  The 3D slab tiles keep one element per round (R = 1): the batch's
// registers pushed the config-5 slab Jv (k_st3l at its 128-VGPR cap) into a spill reload inside the march.
constexpr int kXchgRound = 2, kXchgRoundBlk = 4;

__device__ __forceinline__ uint64_t* halo_flags(uint64_t* base) { return base + kMbWords; }
__device__ __forceinline__ uint64_t* halo_tile_flags(uint64_t* base, int par, int side) {
    return base + kMbWords + (size_t)2 * kHaloSides * kHaloBlocks + (size_t)(par * kHaloSides + side) * kHaloTileFlags;
}
__device__ __forceinline__ uint64_t* halo_inbox(uint64_t* base, int par, int side, int64_t cap) {
    return base + kMbWords + kHaloFlagWords + (size_t)(par * kHaloSides + side) * (size_t)cap;
}
// one lane's wait for a peer's flag to reach `epoch` (bounded: an error at the next host sync, never a hang).
// Exchanges poll their flags in parallel, one lane each: every poll is a system-scope round trip.
__device__ __forceinline__ bool flag_wait(const uint64_t* f, uint64_t epoch) {
    unsigned spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
        if (++spins > g_mb.spin_limit ||
            ((spins & 255) == 0 && __hip_atomic_load(g_mb.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))) {
            __hip_atomic_store(g_mb.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return false;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    return true;
}
__device__ __forceinline__ double ld_inbox(const uint64_t* p) {
    return __longlong_as_double((long long)__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
}

// Ghost patch of one stencil tile through the peers' inboxes, inside the stencil launch (no
// separate exchange kernel): a tile whose rows reach the slab's lower (upper) end pushes its patch
// of my first (last) plane of v -- rows [ra, rb) x columns [ca, cb) of the plane -- into that
// neighbour's inbox (system-scope stores, drained), raises its tile flag there, then waits for the
// neighbour's flag of the same tile; its ghost loads then read the neighbour's patch from my inbox.
// Every other tile never waits, so the exchange overlaps the interior of the stencil.
struct HaloTile {
    int lo, hi;          // this tile needs the lower / upper neighbour's patch
};
template <int R = kXchgRound>
__device__ __forceinline__ bool halo_tile_exchange(const double* __restrict__ v, int64_t plane, int64_t nplanes,
                                                   int64_t nx, int64_t ra, int64_t rb, int64_t ca, int64_t cb, int tile,
                                                   HaloTile t, uint64_t epoch, int64_t cap, int nthreads) {
    __shared__ int hx_ok;
    const int rank = g_mb.rank, nr = g_mb.nranks;
    const int par = (int)(epoch & 1);
    const int64_t w = cb - ca, cnt = (rb - ra) * w;
    for (int side = 0; side < 2; ++side) {  // side 0: my first plane -> the lower rank's "from upper" inbox
        if ((side == 0 && !t.lo) || (side == 1 && !t.hi)) continue;
        const int peer = side == 0 ? (rank + nr - 1) % nr : (rank + 1) % nr;  // (modular: a one-rank self ring, kbench)
        const double* src = side == 0 ? v : v + (nplanes - 1) * plane;
        uint64_t* dst = halo_inbox(g_mb.peers[peer], par, side == 0 ? 1 : 0, cap);
        if constexpr (R == 1) {
            for (int64_t q = threadIdx.x; q < cnt; q += nthreads) {
                const int64_t pos = (ra + q / w) * nx + ca + q % w;
                __hip_atomic_store(dst + pos, (uint64_t)__double_as_longlong(src[pos]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        } else {
            for (int64_t q0 = threadIdx.x; q0 < cnt; q0 += (int64_t)R * nthreads) {  // rounds: loads, one wait, stores
                double a[R];
                int64_t pos[R];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int64_t q = q0 + (int64_t)r * nthreads;
                    pos[r] = (ra + q / w) * nx + ca + q % w;
                    a[r] = q < cnt ? src[pos[r]] : 0.0;
                }
                wait_loads();
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if (q0 + (int64_t)r * nthreads < cnt)
                        __hip_atomic_store(dst + pos[r], (uint64_t)__double_as_longlong(a[r]), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every thread drains its stores before the flag
    __syncthreads();
    if (threadIdx.x < 64) {  // lane 0 the lower side, lane 1 the upper: flags raised and polled in parallel
        const int side = (int)threadIdx.x;
        const bool mine = (side == 0 && t.lo) || (side == 1 && t.hi);
        if (mine)
            __hip_atomic_store(halo_tile_flags(g_mb.peers[side == 0 ? (rank + nr - 1) % nr : (rank + 1) % nr], par, side ^ 1) + tile,
                               epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t t0 = wall_clock64();
        const bool ok = !mine || flag_wait(halo_tile_flags(g_mb.self, par, side) + tile, epoch);
        const bool all = __all(ok);
        if (side == 0) {
            hx_ok = all ? 1 : 0;
            wait_note(kWaitHalo, t0);
        }
    }
    __syncthreads();
    return hx_ok != 0;
}

}  // namespace
}  // namespace nk
