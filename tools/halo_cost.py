"""Cost of the ghost-plane exchange on config 5's slab shape, measured on ONE GPU.

Two processes share the GPU, each owning a 512 x 512 x 64 z-slab of 3D heat (G_Euler! ∘ diffusion!,
FD and exact Jv), and time a loop of Jv products (optionally also a fixed-budget GMRES(20) solve, --itmax),
in three modes:

  alone   no communicator: two independent slabs, ghost planes zero -- no exchange at all
  fused   peer mailbox; v's ghost planes travel inside the Jv launch (halo_tile_exchange, the default)
  kernel  peer mailbox; a separate exchange kernel before every Jv (NK_HALO_FUSE=0, kernel-variant build)

Both processes run their kernels concurrently on the one GPU, so absolute times are those of a shared
device; the differences between the modes are the exchange's cost.  Not part of the product.

Usage (GPU box): python tools/halo_cost.py [--nx 512 --ny 512 --nzl 64] [--reps 40] [--itmax 0]
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

ap = argparse.ArgumentParser()
ap.add_argument("--nx", type=int, default=512)
ap.add_argument("--ny", type=int, default=512)
ap.add_argument("--nzl", type=int, default=64, help="planes per rank (config 5: 512 / 8)")
ap.add_argument("--reps", type=int, default=40)
ap.add_argument("--itmax", type=int, default=0,
                help="> 0: also a fixed-budget GMRES(20) solve (two ranks sharing one GPU time out at the config-5 "
                     "slab: their spinning reduction consumers starve each other -- use a smaller --ny)")
ap.add_argument("--modes", default="alone,fused,kernel,alone,fused,kernel")
ap.add_argument("--child", default="")
args = ap.parse_args()


def child(mode):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch.distributed as dist

    import _nkpath  # noqa: F401
    import ariadne_hip as ah

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    ctx = ah.Context(0)
    ah.set_default_context(ctx)
    nx, ny, nzl = args.nx, args.ny, args.nzl
    if mode == "alone":
        grid = ah.Grid.full(nx, ny, nzl)
    else:
        handles = [None] * world
        dist.all_gather_object(handles, ctx.mailbox_handle())
        ctx.mailbox_open(rank, world, b"".join(handles))
        grid = ah.slab((nx, ny, nzl * world), rank, world)
    nz = nzl * world
    rng = np.random.default_rng(11 + rank)
    un = rng.standard_normal(grid.np_shape)
    hx, hy, hz, a = 1.0 / (nx + 1), 1.0 / (ny + 1), 1.0 / (nz + 1), 0.01
    dt = 1.0 / (2.0 * a * (1 / hx ** 2 + 1 / hy ** 2 + 1 / hz ** 2))
    und = ah.DeviceArray.from_numpy(un, grid, ctx)
    F_, p = ah.G_Euler_.bind(ah.diffusion3d_), (und, dt, None, (a, hx, hy, hz, ah.bc_zero_), 0.0)
    u = ah.DeviceArray.from_numpy(un + 0.01 * rng.standard_normal(grid.np_shape), grid, ctx)
    res, out = u.zero(), u.zero()
    v = ah.DeviceArray.from_numpy(rng.standard_normal(grid.np_shape), grid, ctx)
    F_(res, u, p)
    J = ah.JacobianOperator(F_, res, u, p, jv="fd")
    out_rec = dict(mode=mode, rank=rank, path=ctx.path_info())
    for _ in range(3):
        ah.mul_(out, J, v)
    ctx.sync()
    dist.barrier()
    ctx.prof_enable(1)
    t0 = time.perf_counter()
    for _ in range(args.reps):
        ah.mul_(out, J, v)
    ctx.sync()
    out_rec["jv_us"] = (time.perf_counter() - t0) / args.reps * 1e6
    out_rec["jv_prof"] = ctx.prof_read()
    ctx.prof_reset()
    Je = ah.JacobianOperator(F_, res, u, p, jv="exact")
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        ah.mul_(out, Je, v)
    ctx.sync()
    out_rec["jv_exact_us"] = (time.perf_counter() - t0) / args.reps * 1e6
    out_rec["jv_exact_prof"] = ctx.prof_read()
    ctx.prof_reset()
    if args.itmax <= 0:
        dist.barrier()
        print("RESULT " + json.dumps(out_rec), flush=True)
        return
    ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=20))
    ah.krylov_solve_(ws, J, res, atol=0.0, rtol=0.0, itmax=5)  # warm-up (allocations, first launches)
    ctx.sync()
    dist.barrier()
    ctx.prof_reset()
    t0 = time.perf_counter()
    ah.krylov_solve_(ws, J, res, atol=0.0, rtol=0.0, itmax=args.itmax)
    ctx.sync()
    out_rec["gmres_us_per_step"] = (time.perf_counter() - t0) / args.itmax * 1e6
    out_rec["gmres_prof"] = ctx.prof_read()
    out_rec["niter"] = ws.stats.niter
    dist.barrier()
    print("RESULT " + json.dumps(out_rec), flush=True)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def run_mode(mode):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), WORLD_SIZE="2",
               GPU_MAX_HW_QUEUES="1", NK_KBENCH_LIB="1")
    if mode == "kernel":
        env["NK_HALO_FUSE"] = "0"
    else:
        env.pop("NK_HALO_FUSE", None)
    logs, procs = [], []
    for r in range(2):
        f = tempfile.TemporaryFile()
        logs.append(f)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), "--child", mode,
                                       "--nx", str(args.nx), "--ny", str(args.ny), "--nzl", str(args.nzl),
                                       "--reps", str(args.reps), "--itmax", str(args.itmax)],
                                      env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), stdout=f, stderr=subprocess.STDOUT))
    end = time.time() + 240
    while any(q.poll() is None for q in procs):
        if time.time() > end or any(q.returncode not in (None, 0) for q in procs):
            for q in procs:
                if q.poll() is None:
                    q.kill()
            break
        time.sleep(0.2)
    recs = []
    for r, f in enumerate(logs):
        f.seek(0)
        text = f.read().decode(errors="replace")
        lines = [ln for ln in text.splitlines() if ln.startswith("RESULT ")]
        if procs[r].returncode != 0 or not lines:
            print(f"mode {mode} rank {r} failed (rc {procs[r].returncode}):\n{text[-3000:]}", flush=True)
            sys.exit(1)
        recs.append(json.loads(lines[-1][7:]))
    return recs


def summary(recs):
    def cls(key, name):
        vals = [r[key].get(name) for r in recs if r[key].get(name)]
        if not vals:
            return None
        return dict(launches=vals[0]["launches"], avg_us=max(v["ms"] * 1e3 / max(1, v["timed"]) for v in vals))

    def classes(key):
        return {k: cls(key, k) for k in sorted(set().union(*[r.get(key, {}) for r in recs]))}

    return dict(mode=recs[0]["mode"], jv_us=max(r["jv_us"] for r in recs), jv_exact_us=max(r["jv_exact_us"] for r in recs),
                gmres_us_per_step=max(r.get("gmres_us_per_step", 0.0) for r in recs), niter=recs[0].get("niter"),
                halo_in_launch=recs[0]["path"]["halo_in_launch"], mailbox=recs[0]["path"]["mailbox"],
                jv_classes=classes("jv_prof"), jv_exact_classes=classes("jv_exact_prof"), gmres_classes=classes("gmres_prof"))


if args.child:
    child(args.child)
    sys.exit(0)

print(f"halo cost: 2 ranks sharing one GPU, {args.nx} x {args.ny} x {args.nzl} z-slab each (3D heat, G_Euler!, FD Jv)",
      flush=True)
rows = []
for mode in args.modes.split(","):
    s = summary(run_mode(mode))
    rows.append(s)
    print(json.dumps(s), flush=True)
print("\nmode     FD Jv us/Jv  exact Jv us/Jv  GMRES us/step   (wall per call, max over the 2 ranks; the GPU is shared)")
for s in rows:
    print(f"{s['mode']:8s} {s['jv_us']:11.1f}  {s['jv_exact_us']:13.1f}  {s['gmres_us_per_step']:13.1f}   "
          f"in-launch halo {s['halo_in_launch']}")
