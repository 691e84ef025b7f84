// nk_dist.cpp -- multi-GPU slab decomposition over RCCL (one process per GPU, xGMI).
//
// The reference has no distributed path; its halo storage pattern is examples/halovector.jl
// (ghost layer around the interior, filled by bc!).  Here the ghost planes of a slab are the
// neighbour ranks' boundary planes, exchanged with grouped ncclSend/ncclRecv before every stencil
// application, and every inner product is completed by an 8-byte ncclAllReduce (the Arnoldi
// scalars are then replicated on all ranks, as the Hessenberg/Givens work is).
#include <rccl/rccl.h>

#include <cstring>

#include "nk_internal.hpp"

namespace nk {

struct Comm {
    ncclComm_t comm = nullptr;
};

static int rccl_fail(nk_ctx* c, ncclResult_t r, const char* what) {
    return fail(c, NK_E_RCCL, std::string(what) + ": " + ncclGetErrorString(r));
}

int halo_exchange(nk_ctx* c, const nk_problem* p, const double* v) {
    if (!c->comm) return NK_OK;
    Geo g;
    NK_TRY(geometry(c, p, &g));
    double* vv = const_cast<double*>(v);  // only the ghost planes are written
    const size_t pl = (size_t)g.plane;
    const int up = c->rank + 1, dn = c->rank - 1;
    ncclComm_t comm = c->comm->comm;
    if (dn < 0 && up >= c->nranks) return NK_OK;  // a lone slab has only physical boundaries
    ncclResult_t r = ncclSuccess;
    auto chk = [&r](ncclResult_t x) {
        if (r == ncclSuccess) r = x;
    };
    NK_TRY(launch(c, "halo", 16.0 * pl * ((dn >= 0) + (up < c->nranks)), [&] {
        chk(ncclGroupStart());
        if (dn >= 0) {  // my first interior plane -> lower neighbour's upper ghost; its last -> my lower ghost
            chk(ncclSend(vv, pl, ncclFloat64, dn, comm, c->stream));
            chk(ncclRecv(vv - pl, pl, ncclFloat64, dn, comm, c->stream));
        }
        if (up < c->nranks) {
            chk(ncclSend(vv + (size_t)(g.nplanes - 1) * pl, pl, ncclFloat64, up, comm, c->stream));
            chk(ncclRecv(vv + (size_t)g.nplanes * pl, pl, ncclFloat64, up, comm, c->stream));
        }
        chk(ncclGroupEnd());
    }));
    if (r != ncclSuccess) return rccl_fail(c, r, "halo send/recv");
    return NK_OK;
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
    return NK_OK;
}

int nk_dist_free(nk_ctx* c) {
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
