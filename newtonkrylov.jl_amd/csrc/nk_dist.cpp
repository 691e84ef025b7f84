// nk_dist.cpp -- multi-GPU slab decomposition over RCCL (one process per GPU, xGMI).
//
// The reference has no distributed path; its halo storage pattern is examples/halovector.jl
// (ghost layer around the interior, filled by bc!).  Here the ghost planes of a slab are the
// neighbour ranks' boundary planes, exchanged with grouped ncclSend/ncclRecv before every stencil
// application, and every inner product is completed by an 8-byte ncclAllReduce (the Arnoldi
// scalars are then replicated on all ranks, as the Hessenberg/Givens work is).
#include <rccl/rccl.h>

#include <cstring>
#include <vector>

#include "nk_internal.hpp"

namespace nk {

struct Comm {
    ncclComm_t comm = nullptr;
};

static int rccl_fail(nk_ctx* c, ncclResult_t r, const char* what) {
    return fail(c, NK_E_RCCL, std::string(what) + ": " + ncclGetErrorString(r));
}

// bc_periodic! (heat_2D.jl:15-26) along the slab axis makes the slabs a ring: the lone slab wraps
// onto itself (a local copy), rank 0's lower neighbour is rank nranks-1 and vice versa.
int halo_exchange(nk_ctx* c, const nk_problem* p, const double* v) {
    const bool ring = p && p->bc == NK_BC_PERIODIC;
    if (!ring && !c->comm && !c->mb_on) return NK_OK;
    Geo g;
    NK_TRY(geometry(c, p, &g));
    double* vv = const_cast<double*>(v);  // only the ghost planes are written
    if (ring && c->nranks <= 1) return launch_periodic_fill(c, vv, g.plane, g.nplanes);
    if (!c->comm && !c->mb_on) return NK_OK;
    if (c->mb_on && g.plane <= c->halo_cap) return launch_halo_ipc(c, vv, g.plane, g.nplanes, ring);
    if (!c->comm) return fail(c, NK_E_ARG, "ghost plane larger than the IPC inbox (NK_HALO_CAP) and no RCCL communicator");
    const size_t pl = (size_t)g.plane;
    const int n = c->nranks;
    const int up = c->rank + 1 < n ? c->rank + 1 : (ring ? 0 : -1);
    const int dn = c->rank > 0 ? c->rank - 1 : (ring ? n - 1 : -1);
    ncclComm_t comm = c->comm->comm;
    if (dn < 0 && up < 0) return NK_OK;  // a lone slab has only physical boundaries
    ncclResult_t r = ncclSuccess;
    auto chk = [&r](ncclResult_t x) {
        if (r == ncclSuccess) r = x;
    };
    // Posting order matters when both neighbours are the same rank (a ring of two): sends go up
    // then down, receives come from below then above, so the FIFO matching per peer pairs my
    // lower ghost with the neighbour's last plane and my upper ghost with its first.
    NK_TRY(launch(c, "halo_rccl", 16.0 * pl * ((dn >= 0) + (up >= 0)), [&] {
        chk(ncclGroupStart());
        if (up >= 0) chk(ncclSend(vv + (size_t)(g.nplanes - 1) * pl, pl, ncclFloat64, up, comm, c->stream));
        if (dn >= 0) chk(ncclSend(vv, pl, ncclFloat64, dn, comm, c->stream));
        if (dn >= 0) chk(ncclRecv(vv - pl, pl, ncclFloat64, dn, comm, c->stream));
        if (up >= 0) chk(ncclRecv(vv + (size_t)g.nplanes * pl, pl, ncclFloat64, up, comm, c->stream));
        chk(ncclGroupEnd());
    }));
    if (r != ncclSuccess) return rccl_fail(c, r, "halo send/recv");
    return NK_OK;
}

int exchange_un(nk_ctx* c, const nk_problem* p) {
    if (!p || !nk_is_heat(p->kind) || nk_scheme(p->kind) == 0 || !p->un) return NK_OK;
    return halo_exchange(c, p, p->un);
}

int allreduce_scalar(nk_ctx* c, double* dev, int64_t count) {
    if (!c->comm) return NK_OK;
    ncclResult_t r = ncclSuccess;
    NK_TRY(launch(c, "allreduce", 0.0, [&] {
        r = ncclAllReduce(dev, dev, (size_t)count, ncclFloat64, ncclSum, c->comm->comm, c->stream);
    }));
    if (r != ncclSuccess) return rccl_fail(c, r, "ncclAllReduce");
    return NK_OK;
}

// ---------------------------------------------------------------- peer mailbox (one-shot all-reduce)
// Every reduction scalar goes straight from the producing kernel to every rank's mailbox over
// xGMI (nk_kernels.hip: mb_send / mb_recv); RCCL keeps the halo exchange.  Set up collectively at
// nk_dist_init, verified by a self-test whose verdict all ranks agree on; any failure falls back
// to the RCCL all-reduce.
static int mb_alloc(nk_ctx* c) {
    if (c->mb_self) return NK_OK;
    NK_HIP(c, hipSetDevice(c->device));
    const char* hc = getenv("NK_HALO_CAP");  // doubles per inbox plane (default 1M: a 1024^2 3D plane)
    c->halo_cap = (hc && *hc) ? atoll(hc) : ((int64_t)1 << 20);
    const size_t bytes = sizeof(uint64_t) * (kMbWords + kHaloFlagWords) + sizeof(double) * 4 * (size_t)c->halo_cap;
    void* p = nullptr;
    if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained) != hipSuccess)
        return fail(c, NK_E_NOMEM, "mailbox: fine-grained allocation failed");
    NK_HIP(c, hipMemset(p, 0, bytes));
    c->mb_self = static_cast<uint64_t*>(p);
    if (!c->mb_err) {
        int* h = nullptr;
        NK_HIP(c, hipHostMalloc(&h, 4 * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
        h[0] = 0;
        NK_HIP(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&c->mb_err_dev), h, 0));
        c->mb_err = h;
    }
    return NK_OK;
}

static void mb_disable(nk_ctx* c) {
    c->mb_on = false;
    (void)mailbox_bind(c);
    for (void* p : c->mb_opened) (void)hipIpcCloseMemHandle(p);
    c->mb_opened.clear();
    if (c->mb_peers_dev) (void)hipFree(c->mb_peers_dev);
    c->mb_peers_dev = nullptr;
}

void mb_free(nk_ctx* c) {
    mb_disable(c);
    if (c->mb_self) (void)hipFree(c->mb_self);
    c->mb_self = nullptr;
    if (c->mb_err) (void)hipHostFree(c->mb_err);
    c->mb_err = nullptr;
    c->mb_err_dev = nullptr;
}

// open the peers' mailboxes (local: IPC mappings + device table + kernel binding).  busids (optional,
// nranks x 32 chars): each rank's PCI bus id -- a peer on another device must be reachable by
// peer access (xGMI), and every mapping is probed by a host-initiated copy before any kernel
// dereferences it, so a bad mapping disables the mailbox (RCCL fallback) instead of faulting a kernel.
static int mb_open_peers(nk_ctx* c, int rank, int nranks, const char* handles, const char* busids = nullptr) {
    NK_TRY(mb_alloc(c));
    mb_disable(c);
    std::vector<uint64_t*> peers((size_t)nranks);
    // the resident MGS sweep needs every CU of its grid co-resident: with peers on the same device
    // (no bus ids: the mailbox-only transport, made for ranks on one GPU -- all of them count) it is
    // off, unless NK_RES_SHARED=1 (test rigs) gives every rank's sweep grid CUs / (ranks on the GPU)
    const bool shared_ok = env_cfg("NK_RES_SHARED", 0) != 0;
    int share = busids ? 1 : nranks;
    for (int r = 0; r < nranks; ++r) {
        if (r == rank) {
            peers[r] = c->mb_self;
            continue;
        }
        if (busids) {
            char bus[33];
            std::memcpy(bus, busids + 32 * (size_t)r, 32);
            bus[32] = 0;
            int dev = -1;
            if (hipDeviceGetByPCIBusId(&dev, bus) != hipSuccess) {
                mb_disable(c);
                return fail(c, NK_E_HIP, "mailbox: rank " + std::to_string(r) + "'s device is not visible here");
            }
            if (dev == c->device) ++share;
            if (dev != c->device) {
                int can = 0;
                if (hipDeviceCanAccessPeer(&can, c->device, dev) != hipSuccess || !can) {
                    mb_disable(c);
                    return fail(c, NK_E_HIP, "mailbox: no peer access to rank " + std::to_string(r) + "'s device");
                }
            }
        }
        hipIpcMemHandle_t h;
        std::memcpy(&h, handles + 64 * (size_t)r, 64);
        void* p = nullptr;
        if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
            mb_disable(c);
            return fail(c, NK_E_HIP, "mailbox: hipIpcOpenMemHandle failed for rank " + std::to_string(r));
        }
        c->mb_opened.push_back(p);
        uint64_t probe = 0;
        if (hipMemcpy(&probe, p, sizeof(probe), hipMemcpyDeviceToHost) != hipSuccess) {
            (void)hipGetLastError();
            mb_disable(c);
            return fail(c, NK_E_HIP, "mailbox: rank " + std::to_string(r) + "'s mapping cannot be read");
        }
        peers[r] = static_cast<uint64_t*>(p);
    }
    c->res_share = share;
    c->res_ok = share < 2 || shared_ok;
    NK_HIP(c, hipMalloc(reinterpret_cast<void**>(&c->mb_peers_dev), sizeof(uint64_t*) * nranks));
    NK_HIP(c, hipMemcpy(c->mb_peers_dev, peers.data(), sizeof(uint64_t*) * nranks, hipMemcpyHostToDevice));
    *c->mb_err = 0;
    c->mb_on = true;
    return mailbox_bind(c);
}

// a rank whose mailbox is not open still waits out the self-test's timeout on the others: every
// rank reaches the collective verdict, nobody hangs
// one ring exchange of a small 2-plane grid function whose planes hold (rank, plane, index) codes:
// every ghost plane must hold exactly the neighbour's boundary plane
static bool halo_selftest(nk_ctx* c) {
    if (c->nranks < 2) return true;
    constexpr int64_t pl = 300, np = 2;  // 300 doubles: several blocks of the exchange kernel
    double* base = nullptr;
    if (hipMalloc(&base, sizeof(double) * pl * (np + 2)) != hipSuccess) return false;
    std::vector<double> h((size_t)(pl * (np + 2)), -1.0);
    auto code = [](int r, int64_t k, int64_t i) { return 1e6 * (r + 1) + 1e3 * (double)k + (double)i; };
    for (int64_t k = 0; k < np; ++k)
        for (int64_t i = 0; i < pl; ++i) h[(size_t)((k + 1) * pl + i)] = code(c->rank, k, i);
    bool ok = hipMemcpy(base, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice) == hipSuccess &&
              launch_halo_ipc(c, base + pl, pl, np, true) == NK_OK && hipStreamSynchronize(c->stream) == hipSuccess &&
              hipMemcpy(h.data(), base, sizeof(double) * h.size(), hipMemcpyDeviceToHost) == hipSuccess &&
              !*c->mb_err;
    const int lo = (c->rank + c->nranks - 1) % c->nranks, hi = (c->rank + 1) % c->nranks;
    for (int64_t i = 0; ok && i < pl; ++i)
        ok = h[(size_t)i] == code(lo, np - 1, i) && h[(size_t)((np + 1) * pl + i)] == code(hi, 0, i);
    (void)hipFree(base);
    return ok;
}

static int mb_verdict(nk_ctx* c, bool local_ok) {
    bool ok = local_ok;
    if (c->mb_on) {
        bool t = false;
        if (mailbox_selftest(c, &t) != NK_OK) t = false;
        ok = ok && t && halo_selftest(c);  // reductions and ghost planes through the peer mappings
    }
    if (c->comm) {  // all ranks must take the same path: min over ranks
        double v = ok ? 1.0 : 0.0;
        NK_HIP(c, hipMemcpy(c->scal, &v, sizeof(double), hipMemcpyHostToDevice));
        if (ncclAllReduce(c->scal, c->scal, 1, ncclFloat64, ncclMin, c->comm->comm, c->stream) != ncclSuccess) v = 0.0;
        else {
            NK_HIP(c, hipMemcpyAsync(c->hpin, c->scal, sizeof(double), hipMemcpyDeviceToHost, c->stream));
            NK_HIP(c, hipStreamSynchronize(c->stream));
            v = c->hpin[0];
        }
        ok = ok && v == 1.0;
    }
    if (c->mb_err) *c->mb_err = 0;
    if (!ok) {
        mb_disable(c);
        return fail(c, NK_E_RCCL, "peer mailbox self-test failed (values did not arrive)");
    }
    return NK_OK;
}

}  // namespace nk

using namespace nk;

extern "C" {

int nk_dist_unique_id(char out[128]) {
    if (!out) return NK_E_ARG;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return NK_E_RCCL;
    static_assert(sizeof(id.internal) == 128, "ncclUniqueId size");
    std::memcpy(out, id.internal, 128);
    return NK_OK;
}

int nk_dist_init(nk_ctx* c, int32_t rank, int32_t nranks, const char id[128]) {
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return NK_E_ARG;
    if (c->comm) return fail(c, NK_E_STATE, "context already distributed");
    const char* force = getenv("NK_DIST_FORCE");  // 1-rank communicator: exercises the RCCL path on one GPU
    if (nranks == 1 && !(force && *force == '1')) {
        c->rank = 0;
        c->nranks = 1;
        return NK_OK;
    }
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, 128);
    NK_HIP(c, hipSetDevice(c->device));
    Comm* cm = new Comm();
    ncclResult_t r = ncclCommInitRank(&cm->comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        delete cm;
        return rccl_fail(c, r, "ncclCommInitRank");
    }
    c->comm = cm;
    c->rank = rank;
    c->nranks = nranks;
    const char* mbe = getenv("NK_DIST_MAILBOX");
    // one-shot peer all-reduce of the scalars: on by default with several ranks; NK_DIST_MAILBOX=1
    // also turns it on for a forced 1-rank communicator (exercises the path on one GPU), =0 off
    const bool mb_want = (mbe && *mbe == '1') || (nranks > 1 && !(mbe && *mbe == '0'));
    if (mb_want && nranks <= kMbRanks) {
        // per rank: 64-byte IPC handle + 32-byte PCI bus id of its device
        constexpr size_t kRec = 96;
        std::vector<char> all(kRec * nranks, 0);
        // the exchange buffer is the context's reduction scratch (allocated at nk_ctx_create), so no
        // rank can fail an allocation here and leave the others alone in the collectives below
        static_assert(kRec * kMbRanks <= sizeof(double) * kRedCap, "handle records fit one reduction slot");
        char* dbuf = reinterpret_cast<char*>(c->red);
        int rc = nk_dist_mailbox_handle(c, all.data() + kRec * (size_t)rank);
        if (rc == NK_OK && hipDeviceGetPCIBusId(all.data() + kRec * (size_t)rank + 64, 32, c->device) != hipSuccess)
            rc = NK_E_HIP;
        // allgather the IPC handles: collective, every rank takes part whatever its local state
        (void)hipMemcpy(dbuf + kRec * (size_t)rank, all.data() + kRec * (size_t)rank, kRec, hipMemcpyHostToDevice);
        const ncclResult_t ag = ncclAllGather(dbuf + kRec * (size_t)rank, dbuf, kRec, ncclChar, cm->comm, c->stream);
        if (ag != ncclSuccess || hipStreamSynchronize(c->stream) != hipSuccess ||
            hipMemcpy(all.data(), dbuf, all.size(), hipMemcpyDeviceToHost) != hipSuccess)
            rc = NK_E_RCCL;
        if (ag != ncclSuccess) {
            // still join the verdict's all-reduce (the other ranks are in it), then report the failure
            (void)mb_verdict(c, false);
            return rccl_fail(c, ag, "ncclAllGather (mailbox handles)");
        }
        if (rc == NK_OK) {
            std::vector<char> handles(64 * (size_t)nranks), busids(32 * (size_t)nranks);
            for (int r = 0; r < nranks; ++r) {
                std::memcpy(handles.data() + 64 * (size_t)r, all.data() + kRec * (size_t)r, 64);
                std::memcpy(busids.data() + 32 * (size_t)r, all.data() + kRec * (size_t)r + 64, 32);
            }
            rc = mb_open_peers(c, rank, nranks, handles.data(), busids.data());
        }
        if (mb_verdict(c, rc == NK_OK) != NK_OK) {
            std::fprintf(stderr, "[nkhip] rank %d: peer mailbox off (%s); reductions use ncclAllReduce\n", rank,
                         c->err.c_str());
            c->err.clear();
        }
    }
    return NK_OK;
}

int nk_dist_mailbox_handle(nk_ctx* c, char out[64]) {
    if (!c || !out) return NK_E_ARG;
    NK_TRY(mb_alloc(c));
    hipIpcMemHandle_t h;
    NK_HIP(c, hipIpcGetMemHandle(&h, c->mb_self));
    static_assert(sizeof(h) == 64, "hipIpcMemHandle_t size");
    std::memcpy(out, &h, 64);
    return NK_OK;
}

int nk_dist_mailbox_open(nk_ctx* c, int32_t rank, int32_t nranks, const char* handles) {
    if (!c || !handles || nranks < 1 || nranks > kMbRanks || rank < 0 || rank >= nranks) return NK_E_ARG;
    if (c->comm) return fail(c, NK_E_STATE, "nk_dist_init already set up the mailbox of this context");
    c->rank = rank;  // mailbox-only (no RCCL communicator): reductions across ranks, no halo exchange
    c->nranks = nranks;
    const int rc = mb_open_peers(c, rank, nranks, handles);
    return mb_verdict(c, rc == NK_OK);
}

int nk_dist_mailbox_active(nk_ctx* c) { return (c && c->mb_on) ? 1 : 0; }

int nk_dist_path(nk_ctx* c, nk_path_info* out) {
    if (!c || !out) return NK_E_ARG;
    std::memset(out, 0, sizeof(*out));
    out->rank = c->rank;
    out->nranks = c->nranks;
    out->device = c->device;
    out->ranks_on_device = c->res_share;
    out->rccl = c->comm ? 1 : 0;
    out->mailbox = c->mb_on ? 1 : 0;
    // the resident sweep also needs the mailbox when ranks cross (RCCL reductions need the host between passes)
    out->resident_sweep = (c->res_ok && (!c->comm || c->mb_on)) ? 1 : 0;
    out->resident_blocks = c->res_gran ? c->res_blocks : 0;
    out->halo_in_launch = (halo_fuse_knob() && c->mb_on && c->nranks > 1 && c->halo_cap > 0) ? 1 : 0;
    out->mailbox_error = (c->mb_err && *(volatile int*)c->mb_err) ? 1 : 0;
    out->halo_cap = c->halo_cap;
    if (hipDeviceGetPCIBusId(out->pci_bus_id, (int)sizeof(out->pci_bus_id), c->device) != hipSuccess) {
        (void)hipGetLastError();
        out->pci_bus_id[0] = 0;
    }
    return NK_OK;
}

int nk_dist_free(nk_ctx* c) {
    if (c) mb_free(c);
    if (!c || !c->comm) return NK_OK;
    ncclCommDestroy(c->comm->comm);
    delete c->comm;
    c->comm = nullptr;
    c->nranks = 1;
    c->rank = 0;
    return NK_OK;
}

int nk_dist_allreduce_sum(nk_ctx* c, double* dev_buf, int64_t count) {
    if (!c || !dev_buf || count < 0) return NK_E_ARG;
    return allreduce_scalar(c, dev_buf, count);
}

int nk_halo_exchange(nk_ctx* c, const nk_problem* p, double* v) {
    if (!c || !v) return NK_E_ARG;
    return halo_exchange(c, p, v);
}

}  // extern "C"
