"""Worker for the multi-rank GPU test (launched by tests/test_hip_dist.py through torch.distributed.run).

Every rank owns a slab of a 2D Bratu grid, builds its device vectors from the global initial
condition, runs the distributed HIP path (RCCL halo exchange + all-reduced inner products inside
libnkhip.so) and rank 0 writes the gathered solution, one Jv product and the solver stats.
One GPU per rank (LOCAL_RANK) when the box has enough; otherwise the test sets
NK_WORKER_SHARED_DEVICE=1 and all ranks share device 0 (only the mailbox transport can run there:
RCCL refuses two ranks on one device, and only then is its refusal reported as a skip).
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _nkpath  # noqa: F401,E402
import ariadne_hip as ah  # noqa: E402
import torch.distributed as dist  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--out", required=True)
ap.add_argument("--nx", type=int, default=48)
ap.add_argument("--ny", type=int, default=40)
ap.add_argument("--nz", type=int, default=24, help="heat3d: planes of the global grid")
ap.add_argument("--jv", default="exact")
ap.add_argument("--tol-rel", type=float, default=1e-9, help="Newton tol_rel of the Bratu solve")
ap.add_argument("--krylov-itmax", type=int, default=0,
                help="> 0: instead of the Newton solve, one restarted GMRES(10) solve J x = F(u0) with this fixed "
                     "budget (atol = rtol = 0); rank 0 saves x and the residual history")
ap.add_argument("--precond", choices=["none", "ilu0", "jacobi"], default="none",
                help="with --krylov-itmax: right preconditioner N = ilu0(J) (block Jacobi: each slab factored alone); "
                     "jacobi: the Newton solve's N factory (1 ./ diag(J), pointwise: the global operator)")
ap.add_argument("--problem", choices=["bratu", "heat_periodic", "heat3d"], default="bratu",
                help="heat_periodic: G_Trapezoid! ∘ diffusion! with bc_periodic! -- u_n's ghost planes are "
                     "exchanged too and the slabs form a ring (rank 0 <-> rank world-1)")
ap.add_argument("--fault-rank", type=int, default=-1,
                help=">= 0: failure path -- after the first reductions this rank stops taking part (it waits at a "
                     "gloo barrier, its context alive), the others reduce again and must get an NK_E_* error in "
                     "bounded time; rank 0 records each rank's outcome")
ap.add_argument("--pgrid", default="",
                help="heat3d: px,py,pz -- 3D blocks (nk_dist_grid) instead of z-slabs; x / y ghost faces exchanged too")
ap.add_argument("--scheme", choices=["midpoint", "euler", "trapezoid"], default="midpoint",
                help="heat3d: G_Midpoint!(alpha 0.3) or G_Euler! (whose FD Jv recomputes F(u): the F0R kernels)")
ap.add_argument("--check-errors", action="store_true",
                help="with --pgrid: the process grid's refusals (a wrong grid, a grid after allocation, bc_periodic!)")
ap.add_argument("--transport", choices=["rccl", "mailbox"], default="rccl",
                help="rccl: nk_dist_init (RCCL bootstrap, then the peer mailbox / RCCL fallback); mailbox: "
                     "IPC handles exchanged over gloo, no RCCL at all (works with every rank on one GPU)")
args = ap.parse_args()

dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
device = 0 if os.environ.get("NK_WORKER_SHARED_DEVICE") == "1" else int(os.environ.get("LOCAL_RANK", "0"))
ctx = ah.Context(device)
ah.set_default_context(ctx)


def bcast(obj, src):
    box = [obj]
    dist.broadcast_object_list(box, src=src)
    return box[0]


if args.transport == "mailbox":
    handles = [None] * world
    dist.all_gather_object(handles, ctx.mailbox_handle())
    ctx.mailbox_open(rank, world, b"".join(handles))
else:
    try:
        ah.init_distributed(ctx, rank, world, bcast)
    except ah.NKError as e:
        if os.environ.get("NK_WORKER_SHARED_DEVICE") != "1":
            raise  # one GPU per rank: an RCCL failure is a failure
        if rank == 0:
            json.dump({"skip": f"RCCL communicator could not be created: {e}"}, open(args.out + ".json", "w"))
        sys.exit(0)

nx, ny = args.nx, args.ny
if args.problem == "heat3d":  # 3D heat, implicit midpoint, z-slabs (k_st3l: the ghost planes travel in the stencil)
    nz = args.nz
    if args.pgrid:  # 3D blocks: every vector allocated after the process grid carries its x / y faces
        pg = tuple(int(t) for t in args.pgrid.split(","))
        early = None
        if args.check_errors:  # a vector allocated BEFORE the process grid (no faces), and a wrong grid
            early = ah.DeviceArray(ah.block((nx, ny, nz), rank, pg), ctx)
            errs = {}
            try:
                ctx.set_process_grid(world + 1, 1, 1)
            except ah.NKError as e:
                errs["wrong_grid"] = str(e)
            try:
                ctx.set_process_grid(*pg)  # vectors exist: switching to blocks now is refused
            except ah.NKError as e:
                errs["after_alloc"] = str(e)
            early.free()
        ctx.set_process_grid(*pg)
        grid = ah.block((nx, ny, nz), rank, pg)
        if args.check_errors:
            hx, hy, hz, a = 1.0 / (nx + 1), 1.0 / (ny + 1), 1.0 / (nz + 1), 0.01
            un0 = ah.DeviceArray(grid, ctx)
            r0 = un0.zero()
            try:  # bc_periodic! keeps z-slabs
                ah.G_Euler_.bind(ah.diffusion3d_)(r0, un0, (un0, 1e-3, None, (a, hx, hy, hz, ah.bc_periodic_), 0.0))
                ctx.sync()
            except ah.NKError as e:
                errs["periodic"] = str(e)
            outs = [None] * world
            dist.all_gather_object(outs, errs)
            if rank == 0:
                json.dump(dict(errors=outs, world=world), open(args.out + ".json", "w"))
            dist.barrier()
            ctx.sync()
            sys.exit(0)
    else:
        grid = ah.slab((nx, ny, nz), rank, world)
    x0, y0, z0 = grid.origin or (0, 0, grid.offset)
    nxl, nyl, nzl = grid.shape_xyz
    sl = (slice(z0, z0 + nzl), slice(y0, y0 + nyl), slice(x0, x0 + nxl))
    rng = np.random.default_rng(9)
    un_glob = rng.standard_normal((nz, ny, nx))
    u_glob = un_glob + 0.01 * rng.standard_normal((nz, ny, nx))
    v_glob = rng.standard_normal((nz, ny, nx))
    hx, hy, hz, a = 1.0 / (nx + 1), 1.0 / (ny + 1), 1.0 / (nz + 1), 0.01
    dt = 1.0 / (2.0 * a * (1 / hx ** 2 + 1 / hy ** 2 + 1 / hz ** 2))
    und = ah.DeviceArray.from_numpy(np.ascontiguousarray(un_glob[sl]), grid, ctx)
    G = {"euler": ah.G_Euler_, "trapezoid": ah.G_Trapezoid_}.get(args.scheme) or ah.G_Midpoint_(alpha=0.3)
    F_, p = G.bind(ah.diffusion3d_), (und, dt, None, (a, hx, hy, hz, ah.bc_zero_), 0.0)
    u = ah.DeviceArray.from_numpy(np.ascontiguousarray(u_glob[sl]), grid, ctx)
    res = u.zero()
    vd = ah.DeviceArray.from_numpy(np.ascontiguousarray(v_glob[sl]), grid, ctx)
    out = u.zero()
    F_(res, u, p)
    if args.fault_rank >= 0:  # a rank that stops exchanging: the others' next ghost-face exchange must fail
        import time

        outcome = dict(rank=rank, skipped=rank == args.fault_rank)
        if rank != args.fault_rank:
            t0 = time.perf_counter()
            try:
                F_(res, u, p)  # its exchange waits for the faulty rank's faces
                ctx.sync()
                outcome["error"] = None
            except ah.NKError as e:
                outcome["error"] = str(e)
            outcome["seconds"] = time.perf_counter() - t0
            outcome["path"] = ctx.path_info()
        outs = [None] * world
        dist.all_gather_object(outs, outcome)
        if rank == 0:
            json.dump(dict(fault=outs, world=world), open(args.out + ".json", "w"))
        dist.barrier()
        sys.exit(0)  # no ctx.sync(): the mailbox error is sticky on the ranks that timed out
    if args.krylov_itmax > 0:  # one restarted FD-GMRES(20) solve J x = F(u0), fixed budget
        ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=20))
        J = ah.JacobianOperator(F_, res, u, p, jv="fd")
        ah.krylov_solve_(ws, J, res, restart=True, atol=0.0, rtol=0.0, itmax=args.krylov_itmax, history=True)
        parts = [None] * world
        dist.all_gather_object(parts, dict(sl=sl, x=ws.x.to_numpy(), F=res.to_numpy(), path=ctx.path_info()))
        if rank == 0:
            full = {}
            for key in ("x", "F"):
                full[key] = np.full((nz, ny, nx), np.nan)
                for d in parts:
                    full[key][d["sl"]] = d[key]
            np.savez(args.out + ".npz", h=np.array(ws.stats.residuals), **full)
            json.dump(dict(niter=ws.stats.niter, n_matvec=ws.stats.n_matvec, world=world, path=ctx.path_info(),
                           paths=[d["path"] for d in parts], planes=[d["sl"][0].stop - d["sl"][0].start for d in parts]),
                      open(args.out + ".json", "w"))
        dist.barrier()
        ctx.sync()
        sys.exit(0)
    ah.mul_(out, ah.JacobianOperator(F_, res, u, p, jv="exact"), vd)
    jv_ex = out.to_numpy()
    ah.mul_(out, ah.JacobianOperator(F_, res, u, p, jv="fd"), vd, eps=1e-6)
    jv_fd = out.to_numpy()
    F_loc = res.to_numpy()
    u, r = ah.newton_krylov_(F_, u, p, res, tol_abs=6e-6, jv="fd")
    parts = [None] * world
    dist.all_gather_object(parts, dict(sl=sl, u=u.to_numpy(), jv=jv_ex, jvfd=jv_fd, F=F_loc))
    if rank == 0:
        full = {}
        for key in ("u", "jv", "jvfd", "F"):
            full[key] = np.full((nz, ny, nx), np.nan)
            for d in parts:
                full[key][d["sl"]] = d[key]
        np.savez(args.out + ".npz", **full)
        json.dump(dict(solved=bool(r.solved), outer=r.stats.outer_iterations, inner=r.stats.inner_iterations,
                       world=world, mailbox=ctx.mailbox_active, path=ctx.path_info()), open(args.out + ".json", "w"))
    dist.barrier()
    ctx.sync()
    sys.exit(0)
grid = ah.slab((nx, ny), rank, world)
hx, hy, lam = 1.0 / (nx + 1), 1.0 / (ny + 1), 3.51382
xs = np.arange(1, nx + 1) * hx
y0, nyl = grid.offset, grid.shape_xyz[1]
ys = np.arange(y0 + 1, y0 + nyl + 1) * hy
v_glob = np.random.default_rng(7).standard_normal((ny, nx))
if args.problem == "bratu":
    u0 = np.sin(np.pi * ys)[:, None] * np.sin(np.pi * xs)[None, :]
    F_, p = ah.bratu2d_, (hx, hy, lam)
    kw = dict(memory=10, tol_rel=args.tol_rel, krylov_kwargs=dict(restart=True))
    if args.precond == "jacobi":
        kw["N"] = ah.jacobi
else:
    rng = np.random.default_rng(5)
    un_glob = rng.standard_normal((ny, nx))
    u_glob = un_glob + 0.01 * rng.standard_normal((ny, nx))
    u0 = np.ascontiguousarray(u_glob[y0:y0 + nyl])
    a = 0.01
    dt = hx ** 2 * hy ** 2 / (2.0 * a * (hx ** 2 + hy ** 2))
    und = ah.DeviceArray.from_numpy(np.ascontiguousarray(un_glob[y0:y0 + nyl]), grid, ctx)
    F_, p = ah.heat2d_trapezoid_, (und, dt, None, (a, hx, hy, ah.bc_periodic_), 0.0)
    kw = dict(tol_abs=6e-6, krylov_kwargs=dict(reorthogonalization=True))

u = ah.DeviceArray.from_numpy(u0, grid, ctx)
res = u.zero()
vd = ah.DeviceArray.from_numpy(np.ascontiguousarray(v_glob[y0:y0 + nyl]), grid, ctx)
out = u.zero()
F_(res, u, p)
ah.mul_(out, ah.JacobianOperator(F_, res, u, p, jv=args.jv), vd)
jv_loc = out.to_numpy()
F_loc = res.to_numpy()
ah.mul_(out, ah.JacobianOperator(F_, res, u, p, jv="fd"), vd, eps=1e-7)  # a given eps: bit-comparable
jvfd_loc = out.to_numpy()
dot = ah.kdot(len(u), u, vd)
if args.fault_rank >= 0:
    import time

    outcome = dict(rank=rank, skipped=rank == args.fault_rank)
    if rank != args.fault_rank:
        t0 = time.perf_counter()
        try:
            ah.kdot(len(u), u, vd)  # a reduction the faulty rank never contributes to
            outcome["error"] = None
        except ah.NKError as e:
            outcome["error"] = str(e)
        outcome["seconds"] = time.perf_counter() - t0
        outcome["path"] = ctx.path_info()
    outs = [None] * world
    dist.all_gather_object(outs, outcome)  # the faulty rank joins here: its context stayed alive meanwhile
    if rank == 0:
        json.dump(dict(fault=outs, world=world, first_dot=dot), open(args.out + ".json", "w"))
    dist.barrier()
    sys.exit(0)  # no ctx.sync(): the mailbox error is sticky on the ranks that timed out
if args.krylov_itmax > 0:
    ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=10))
    ctx.prof_enable(1)
    J = ah.JacobianOperator(F_, res, u, p, jv=args.jv)
    N = ah.ilu0(J) if args.precond == "ilu0" else None
    ah.krylov_solve_(ws, J, res, restart=True, atol=0.0, rtol=0.0, itmax=args.krylov_itmax, history=True, N=N)
    sweeps = ctx.prof_read().get("mgs_sweep", {}).get("launches", 0)  # resident sweeps that ran
    ctx.prof_enable(0)
    parts = [None] * world
    dist.all_gather_object(parts, dict(y0=y0, x=ws.x.to_numpy(), F=F_loc, jvfd=jvfd_loc))
    if rank == 0:
        parts.sort(key=lambda d: d["y0"])
        cat = lambda key: np.concatenate([d[key] for d in parts])  # noqa: E731
        np.savez(args.out + ".npz", x=cat("x"), F=cat("F"), jvfd=cat("jvfd"), v=v_glob, h=np.array(ws.stats.residuals))
        json.dump(dict(niter=ws.stats.niter, n_matvec=ws.stats.n_matvec, world=world, sweeps=sweeps,
                       path=ctx.path_info()), open(args.out + ".json", "w"))
    dist.barrier()
    ctx.sync()
    sys.exit(0)
u, r = ah.newton_krylov_(F_, u, p, res, jv=args.jv, **kw)
parts = [None] * world
dist.all_gather_object(parts, dict(y0=y0, u=u.to_numpy(), jv=jv_loc, F=F_loc, jvfd=jvfd_loc))
if rank == 0:
    parts.sort(key=lambda d: d["y0"])
    np.savez(args.out + ".npz", u=np.concatenate([d["u"] for d in parts]), jv=np.concatenate([d["jv"] for d in parts]),
             F=np.concatenate([d["F"] for d in parts]), jvfd=np.concatenate([d["jvfd"] for d in parts]), v=v_glob)
    json.dump(dict(solved=bool(r.solved), outer=r.stats.outer_iterations, inner=r.stats.inner_iterations,
                   n_res=r.stats.n_res, dot=dot, world=world, path=ctx.path_info()), open(args.out + ".json", "w"))
dist.barrier()
ctx.sync()
