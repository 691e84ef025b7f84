"""Multi-GPU setup: one process per GPU, slab decomposition along the slowest axis (nk_dist.cpp), or
3D blocks for the 3D kinds (`block` + Context.set_process_grid: x / y ghost faces as well).

torch.distributed (gloo) is only the control plane here: it broadcasts RCCL's unique id from rank 0.
RCCL then bootstraps the data path: at nk_dist_init the ranks allgather the IPC handles of each
other's peer mailboxes (fine-grained device memory), map them over xGMI and self-test them.  From
then on every inner product is all-reduced through the mailboxes inside the consuming kernel, and
v's ghost planes travel inside the Krylov Jv launch -- no collective per reduction.
RCCL send/recv + ncclAllReduce on the library stream remain the fallback when the mailbox cannot
come up (a peer device invisible to the process, a failed self-test, NK_DIST_MAILBOX=0) and for
ghost planes larger than the inbox.  ctx.path_info() reports which path ran, from launch counts.
"""
from __future__ import annotations

import ctypes as C

from ._lib import NKError, load
from .device import Context, Grid


def dist_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    if load().nk_dist_unique_id(buf) != 0:
        raise NKError("ncclGetUniqueId failed")
    return buf.raw


def slab(global_xyz, rank: int, nranks: int) -> Grid:
    """Split the slowest axis into `nranks` contiguous slabs (sizes differ by at most one plane)."""
    g = tuple(int(d) for d in global_xyz)
    nslow = g[-1]
    if nslow < nranks:
        raise ValueError("fewer planes than ranks")
    base, extra = divmod(nslow, nranks)
    sizes = [base + (1 if r < extra else 0) for r in range(nranks)]
    off = sum(sizes[:rank])
    return Grid(g[:-1] + (sizes[rank],), g, off)


def _split(n: int, parts: int):
    if n < parts:
        raise ValueError("fewer points than ranks along an axis")
    base, extra = divmod(n, parts)
    sizes = [base + (1 if r < extra else 0) for r in range(parts)]
    return sizes, [sum(sizes[:r]) for r in range(parts)]


def block(global_xyz, rank: int, pgrid) -> Grid:
    """The 3D block of `rank` in a px x py x pz process grid (Context.set_process_grid; rank =
    (iz py + iy) px + ix): every axis split like `slab` splits z, so the blocks sharing a face share its
    extents.  pgrid (1, 1, nranks) is `slab`."""
    g = tuple(int(d) for d in global_xyz)
    px, py, pz = (int(d) for d in pgrid)
    if len(g) != 3:
        raise ValueError("blocks are 3D")
    if not 0 <= rank < px * py * pz:
        raise ValueError("rank outside the process grid")
    idx = (rank % px, (rank // px) % py, rank // (px * py))
    shape, origin = [], []
    for d, parts in enumerate((px, py, pz)):
        sizes, offs = _split(g[d], parts)
        shape.append(sizes[idx[d]])
        origin.append(offs[idx[d]])
    return Grid(tuple(shape), g, origin[2], tuple(origin))


def init_distributed(ctx: Context, rank: int, nranks: int, broadcast_object) -> None:
    """Create the RCCL communicator of `ctx`; `broadcast_object(obj, src)` returns rank 0's object
    (e.g. built on torch.distributed.broadcast_object_list)."""
    uid = dist_unique_id() if rank == 0 else None
    uid = broadcast_object(uid, 0)
    ctx.init_distributed(rank, nranks, uid)
