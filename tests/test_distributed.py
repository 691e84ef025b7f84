"""Multi-rank protocol of the slab and 3D-block decompositions, on CPU with gloo (world_size 2, 3 and 8: the driver's node size).

libnkhip.so's distributed path (nk_dist.cpp) does exactly two things beyond the single-GPU code:
before every stencil application it fills the two ghost planes of the input vector with the
neighbouring slabs' boundary planes (RCCL send/recv), and it completes every inner product with a
sum over ranks (RCCL all-reduce) before any consumer reads it.  Its kernels cannot run here, so
this test drives the SAME protocol -- the product's own slab partition (ariadne_hip.slab), ghost
planes filled by gloo send/recv from the neighbours, all-reduced dots -- around a numpy stand-in
for the stencil kernels, and checks it reproduces the single-domain CPU oracle: residuals, Jv,
the GMRES(10) history, and the converged Newton iterate.  (The RCCL plumbing itself is checked on
the GPU box by tests/test_hip_dist.py.)
"""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import _nkpath  # noqa: F401
import ariadne_hip as ah
from oracle import ariadne_ref as ar
from oracle import oracle as oc

NX, NY = 20, 17


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class Slab:
    """One rank's slab with ghost rows, exchanged like nk_dist.cpp halo_exchange."""

    def __init__(self, rank, world):
        self.rank, self.world = rank, world
        self.grid = ah.slab((NX, NY), rank, world)
        self.y0, self.nyl = self.grid.offset, self.grid.shape_xyz[1]
        self.hx, self.hy, self.lam = 1.0 / (NX + 1), 1.0 / (NY + 1), oc.LAMBDA_BRATU

    def padded(self, a):
        """Interior rows + ghost rows from the neighbours (zero on the physical boundary)."""
        pad = np.zeros((self.nyl + 2, NX))
        pad[1:-1] = a
        reqs = []
        lo = torch.zeros(NX, dtype=torch.float64)
        hi = torch.zeros(NX, dtype=torch.float64)
        if self.rank > 0:  # my first plane -> lower neighbour's upper ghost; its last -> my lower ghost
            reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(a[0])), self.rank - 1))
            reqs.append(dist.irecv(lo, self.rank - 1))
        if self.rank < self.world - 1:
            reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(a[-1])), self.rank + 1))
            reqs.append(dist.irecv(hi, self.rank + 1))
        for r in reqs:
            r.wait()
        pad[0], pad[-1] = lo.numpy(), hi.numpy()
        return pad

    def lap(self, a):
        p = self.padded(a)
        c = p[1:-1]
        e = np.pad(c, ((0, 0), (0, 1)))[:, 1:]
        w = np.pad(c, ((0, 0), (1, 0)))[:, :-1]
        return ((e - 2.0 * c) + w) / (self.hx * self.hx) + ((p[2:] - 2.0 * c) + p[:-2]) / (self.hy * self.hy)

    def residual(self, u):
        return self.lap(u) + self.lam * np.exp(u)

    def jv(self, u, v):
        return self.lap(v) + self.lam * (np.exp(u) * v)

    def dot(self, x, y):
        t = torch.tensor([float(np.sum(x * y))], dtype=torch.float64)
        dist.all_reduce(t)
        return float(t.item())


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    S = Slab(rank, world)
    P = oc.bratu2d(NX, NY)
    U0 = oc.sin_ic(P)
    u0 = U0[S.y0:S.y0 + S.nyl].copy()
    v = np.random.default_rng(3).standard_normal((NY, NX))[S.y0:S.y0 + S.nyl]
    F = S.residual(u0)
    Jv = S.jv(u0, v)
    shape = u0.shape
    A = lambda x: S.jv(u0, x.reshape(shape)).ravel()
    kw = dict(memory=10, restart=True, atol=0.0, rtol=1e-10, itmax=60, dot=lambda a, b: S.dot(a, b), n=NX * NY)
    x, st, hist = ar.gmres(A, F.ravel(), **kw)
    # inexact Newton (src/Ariadne.jl:288-372) on the slabs with EW forcing
    ew = ar.EisenstatWalker()
    u = u0.copy()
    res = S.residual(u)
    n_res = math.sqrt(S.dot(res, res))
    tol = 1e-9 * n_res + 1e-12
    eta, outer, inner = ew.initial(), 0, 0
    while n_res > tol and outer <= 50:
        uu = u.copy()
        d, kst, _ = ar.gmres(lambda z: S.jv(uu, z.reshape(shape)).ravel(), res.ravel(), memory=10, restart=True,
                             rtol=eta, dot=lambda a, b: S.dot(a, b), n=NX * NY)
        u = u - d.reshape(shape)
        prior, res = n_res, S.residual(u)
        n_res = math.sqrt(S.dot(res, res))
        eta = ew(eta, tol, n_res, prior)
        outer, inner = outer + 1, inner + kst.niter
    parts = [None] * world
    dist.all_gather_object(parts, dict(y0=S.y0, F=F, Jv=Jv, x=x.reshape(shape), u=u))
    if rank == 0:
        parts.sort(key=lambda d: d["y0"])
        np.savez(out, **{k: np.concatenate([d[k] for d in parts]) for k in ("F", "Jv", "x", "u")},
                 hist=np.array(hist), niter=st.niter, outer=outer, inner=inner)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_slab_protocol_matches_single_domain(tmp_path, world):
    out = str(tmp_path / "dist.npz")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    d = np.load(out)
    P = oc.bratu2d(NX, NY)
    U0 = oc.sin_ic(P)
    v = np.random.default_rng(3).standard_normal((NY, NX))
    F = oc.residual(P, U0)
    assert np.max(np.abs(d["F"] - F)) <= 1e-12 * np.max(np.abs(F))
    assert np.max(np.abs(d["Jv"] - oc.jv_exact(P, U0, v))) <= 1e-12 * np.max(np.abs(d["Jv"]))
    xo, sto, ho = oc.krylov_solve(P, U0, F, memory=10, restart=True, atol=0.0, rtol=1e-10, itmax=60)
    assert int(d["niter"]) == sto["niter"]
    assert np.allclose(d["hist"][:11], ho[:11], rtol=1e-9)
    assert np.max(np.abs(d["x"] - xo)) <= 1e-7 * np.max(np.abs(xo))
    uo, so = oc.newton_krylov(P, U0, memory=10, restart=True, tol_rel=1e-9)
    assert (int(d["outer"]), int(d["inner"])) == (so["outer_iterations"], so["inner_iterations"])
    assert np.max(np.abs(d["u"] - uo)) <= 1e-9 * np.max(np.abs(uo))


# ----------------------------------------------------------------------------- bc_periodic! ring
def ring_padded(a, rank, world):
    """Ghost rows of a periodic slab ring, posted in nk_dist.cpp's halo_exchange order (sends up then
    down, receives from below then above): with two ranks both neighbours are the same rank, and only
    this order pairs my lower ghost with the neighbour's last row under per-peer FIFO matching."""
    up, dn = (rank + 1) % world, (rank - 1) % world
    lo = torch.zeros(a.shape[1], dtype=torch.float64)
    hi = torch.zeros(a.shape[1], dtype=torch.float64)
    reqs = [dist.isend(torch.from_numpy(np.ascontiguousarray(a[-1])), up),
            dist.isend(torch.from_numpy(np.ascontiguousarray(a[0])), dn),
            dist.irecv(lo, dn), dist.irecv(hi, up)]
    for r in reqs:
        r.wait()
    return np.concatenate([lo.numpy()[None], a, hi.numpy()[None]])


def _ring_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = ah.slab((NX, NY), rank, world)
    y0, nyl = g.offset, g.shape_xyz[1]
    rng = np.random.default_rng(5)
    un_g = rng.standard_normal((NY, NX))
    u_g = un_g + 0.01 * rng.standard_normal((NY, NX))
    P = oc.heat2d_euler(NX, NY, scheme="trapezoid", bc=oc.BC_PERIODIC)

    def lap(a):  # diffusion!'s sum with the x wrap in-row and the y wrap through the ring ghosts
        p = ring_padded(a, rank, world)
        c = p[1:-1]
        e, w = np.roll(c, -1, axis=1), np.roll(c, 1, axis=1)
        return ((e - 2.0 * c) + w) / (P.hx * P.hx) + ((p[2:] - 2.0 * c) + p[:-2]) / (P.hy * P.hy)

    un, u = un_g[y0:y0 + nyl], u_g[y0:y0 + nyl]
    G = (un + (P.dt / 2.0) * (P.a * lap(un) + P.a * lap(u))) - u  # implicit.jl:29-37
    parts = [None] * world
    dist.all_gather_object(parts, dict(y0=y0, G=G))
    if rank == 0:
        parts.sort(key=lambda d: d["y0"])
        np.savez(out, G=np.concatenate([d["G"] for d in parts]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_periodic_ring_protocol(tmp_path, world):
    out = str(tmp_path / "ring.npz")
    mp.spawn(_ring_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    rng = np.random.default_rng(5)
    un = rng.standard_normal((NY, NX))
    u = un + 0.01 * rng.standard_normal((NY, NX))
    P = oc.heat2d_euler(NX, NY, un=un, scheme="trapezoid", bc=oc.BC_PERIODIC)
    assert np.array_equal(np.load(out)["G"], oc.residual(P, u))


# ----------------------------------------------------------------------------- 3D blocks (config 5)
NB = (13, 10, 9)  # global nx, ny, nz: uneven splits on every axis


def block_padded(a, pg, rank):
    """One rank's block + one ghost layer on every side, exchanged like nk_dist.cpp's k_faces_ipc: the six
    boundary layers (x faces gathered) to the neighbours of the px x py x pz grid, rank = (iz py + iy) px
    + ix as block_nbr numbers them; zero on the physical boundary."""
    px, py, pz = pg
    ix, iy, iz = rank % px, (rank // px) % py, rank // (px * py)
    nz, ny, nx = a.shape
    pad = np.zeros((nz + 2, ny + 2, nx + 2))
    pad[1:-1, 1:-1, 1:-1] = a
    # (numpy axis, lower / upper side, neighbour or None): z, y, x
    sides = [(0, 0, rank - px * py if iz > 0 else None), (0, 1, rank + px * py if iz + 1 < pz else None),
             (1, 0, rank - px if iy > 0 else None), (1, 1, rank + px if iy + 1 < py else None),
             (2, 0, rank - 1 if ix > 0 else None), (2, 1, rank + 1 if ix + 1 < px else None)]
    reqs, got = [], []
    for ax, hi, nbr in sides:
        if nbr is None:
            continue
        layer = np.ascontiguousarray(np.take(a, -1 if hi else 0, axis=ax))
        recv = torch.zeros(layer.shape, dtype=torch.float64)
        reqs.append(dist.isend(torch.from_numpy(layer), nbr))
        reqs.append(dist.irecv(recv, nbr))
        got.append((ax, hi, recv))
    for r in reqs:
        r.wait()
    for ax, hi, recv in got:
        idx = [slice(1, -1)] * 3
        idx[ax] = -1 if hi else 0
        pad[tuple(idx)] = recv.numpy()
    return pad


def _block_worker(rank, world, port, out, pg):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = ah.block(NB, rank, pg)
    (x0, y0, z0), (nxl, nyl, nzl) = g.origin, g.shape_xyz
    sl = (slice(z0, z0 + nzl), slice(y0, y0 + nyl), slice(x0, x0 + nxl))
    rng = np.random.default_rng(4)
    un, u, v = (rng.standard_normal(NB[::-1]) for _ in range(3))
    G = oc.heat3d_euler(*NB, un=un, scheme="midpoint", alpha=0.3)  # the global spacing and time step
    # the stencil stand-in: the oracle on the padded block, its inner points kept (the ring holds the
    # neighbours' layers, or the Dirichlet zeros)
    upad, unpad, vpad = (block_padded(np.ascontiguousarray(w[sl]), pg, rank) for w in (u, un, v))
    P = oc.Problem(G.kind, nxl + 2, nyl + 2, nzl + 2, hx=G.hx, hy=G.hy, hz=G.hz, a=G.a, dt=G.dt, un=unpad,
                   alpha=G.alpha)
    F = oc.residual(P, upad)[1:-1, 1:-1, 1:-1]
    Jv = oc.jv_exact(P, upad, vpad)[1:-1, 1:-1, 1:-1]
    t = torch.tensor([float(np.sum(F * F))], dtype=torch.float64)
    dist.all_reduce(t)
    parts = [None] * world
    dist.all_gather_object(parts, dict(sl=sl, F=F, Jv=Jv))
    if rank == 0:
        full = {k: np.full(NB[::-1], np.nan) for k in ("F", "Jv")}
        for d in parts:
            for k in full:
                full[k][d["sl"]] = d[k]
        np.savez(out, nrm2=float(t.item()), **full)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("pg", [(2, 1, 1), (1, 2, 2), (2, 2, 2), (3, 1, 2)])
def test_block_protocol_matches_single_domain(tmp_path, pg):
    """The 3D-block protocol (ah.block's partition, block_nbr's rank numbering, six faces per exchange)
    around the oracle's heat stencil (G_Midpoint!, alpha 0.3): residual and exact JVP of every block,
    assembled, bit for bit the single-domain oracle's; the all-reduced ||F||^2 to rounding."""
    world = int(np.prod(pg))
    out = str(tmp_path / "blk.npz")
    mp.spawn(_block_worker, args=(world, _free_port(), out, pg), nprocs=world, join=True)
    d = np.load(out)
    rng = np.random.default_rng(4)
    un, u, v = (rng.standard_normal(NB[::-1]) for _ in range(3))
    P = oc.heat3d_euler(*NB, un=un, scheme="midpoint", alpha=0.3)
    F = oc.residual(P, u)
    np.testing.assert_array_equal(d["F"], F)
    np.testing.assert_array_equal(d["Jv"], oc.jv_exact(P, u, v))
    assert abs(float(d["nrm2"]) - float(np.sum(F * F))) <= 1e-12 * float(np.sum(F * F))
