"""Cost of the ghost-plane exchange in a config-5 Krylov solve, measured on ONE GPU with ONE process
(VERDICT r02 item 6): a forced one-rank communicator over the peer mailbox whose lone rank is its own
lower and upper neighbour (kbench NK_HALO_SELF=1) -- a self ring that runs the exchange of every Jv
(push the boundary patches, raise the flags, wait, read the inbox) without a second process competing
for the GPU.  Modes, each in its own process:

  plain   no communicator: ghost planes zero, no exchange, local reductions
  mbox    forced one-rank mailbox, no exchange (every reduction scalar through the mailbox)
  fused   + self ring, v's ghost planes inside the Jv launch (halo_tile_exchange, the product default)
  kernel  + self ring, a separate exchange kernel before every Jv (NK_HALO_FUSE=0)
  blocks  3D only: the rank is its own neighbour on all SIX sides (NK_HALO_SELF=2) -- config 5's 3D-block
          path: one packed-face exchange launch per Jv (k_faces_ipc) and k_st3l reading the x / y faces
          at the block's edges (the operator differs: every axis wraps; the cost is what is measured)
  blocki  the same with every ghost layer of v inside the Jv launch (blk_tile_exchange, NK_BLK_INLAUNCH=1)

fused - mbox and kernel - mbox are the exchange's cost per Arnoldi step.  fused and kernel apply the same
operator (the same ghost planes, the same per-point arithmetic) but the fused launch dispatches the
slab-end tiles first, so its block partials of <V_1, Jv> are summed in another order: their solutions
agree to rounding (reported), not bit for bit.  Not part of the product.

Usage (GPU box): python tools/halo_self.py [--nx 512 --ny 512 --nz 64] [--itmax 60]
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

ap = argparse.ArgumentParser()
ap.add_argument("--nx", type=int, default=512)
ap.add_argument("--ny", type=int, default=512)
ap.add_argument("--nz", type=int, default=64, help="planes of the slab (config 5: 512 / 8); 0: a 2D Bratu slab "
                                                   "of nx x ny (ghost rows in k_st2d's launch)")
ap.add_argument("--itmax", type=int, default=60)
ap.add_argument("--modes", default="plain,mbox,fused,kernel,plain,mbox,fused,kernel")
ap.add_argument("--child", default="")
ap.add_argument("--xdir", default="/tmp", help="where the children leave their solutions")
args = ap.parse_args()

ENV = {
    "plain": {},
    "mbox": {"NK_DIST_FORCE": "1", "NK_DIST_MAILBOX": "1"},
    "fused": {"NK_DIST_FORCE": "1", "NK_DIST_MAILBOX": "1", "NK_HALO_SELF": "1"},
    "kernel": {"NK_DIST_FORCE": "1", "NK_DIST_MAILBOX": "1", "NK_HALO_SELF": "1", "NK_HALO_FUSE": "0"},
    "blocks": {"NK_DIST_FORCE": "1", "NK_DIST_MAILBOX": "1", "NK_HALO_SELF": "2"},
    "blocki": {"NK_DIST_FORCE": "1", "NK_DIST_MAILBOX": "1", "NK_HALO_SELF": "2", "NK_BLK_INLAUNCH": "1"},
}


def child(mode):
    sys.path.insert(0, ROOT)
    import numpy as np

    import _nkpath  # noqa: F401
    import ariadne_hip as ah

    ctx = ah.Context(0)
    ah.set_default_context(ctx)
    if mode != "plain":
        ctx.init_distributed(0, 1, ah.dist_unique_id())
    nx, ny, nz = args.nx, args.ny, args.nz
    rng = np.random.default_rng(11)
    if nz == 0:  # 2D Bratu slab: the ghost rows travel in k_st2d's launch
        grid = ah.Grid.full(nx, ny)
        hx, hy = 1.0 / (nx + 1), 1.0 / (8 * ny + 1)
        F_, p = ah.bratu2d_, (hx, hy, 3.51382)
        xs, ys = np.arange(1, nx + 1) * hx, np.arange(1, ny + 1) * hy
        u = ah.DeviceArray.from_numpy(np.sin(np.pi * ys)[:, None] * np.sin(np.pi * xs)[None, :], grid, ctx)
    else:
        grid = ah.Grid.full(nx, ny, nz)
        un = rng.standard_normal(grid.np_shape)
        hx, hy, hz, a = 1.0 / (nx + 1), 1.0 / (ny + 1), 1.0 / (8 * nz + 1), 0.01
        dt = 1.0 / (2.0 * a * (1 / hx ** 2 + 1 / hy ** 2 + 1 / hz ** 2))
        und = ah.DeviceArray.from_numpy(un, grid, ctx)
        F_, p = ah.G_Euler_.bind(ah.diffusion3d_), (und, dt, None, (a, hx, hy, hz, ah.bc_zero_), 0.0)
        u = ah.DeviceArray.from_numpy(un + 0.01 * rng.standard_normal(grid.np_shape), grid, ctx)
    res = u.zero()
    F_(res, u, p)
    J = ah.JacobianOperator(F_, res, u, p, jv="fd")
    ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=20))
    kw = dict(restart=True, atol=0.0, rtol=0.0, itmax=args.itmax)
    ah.krylov_solve_(ws, J, res, **kw)  # warm-up
    ctx.sync()
    ctx.prof_enable(1)
    t0 = time.perf_counter()
    ah.krylov_solve_(ws, J, res, **kw)
    ctx.sync()
    dt_s = time.perf_counter() - t0
    prof = ctx.prof_read()
    ctx.prof_enable(0)
    x = ws.x.to_numpy()
    np.save(os.path.join(args.xdir, f"x_{mode}.npy"), x)
    rec = dict(mode=mode, us_per_step=dt_s / ws.stats.niter * 1e6, n_matvec=ws.stats.n_matvec, niter=ws.stats.niter,
               x_sha=hashlib.sha1(x.tobytes()).hexdigest()[:16], path=ctx.path_info(),
               classes={k: dict(launches=v["launches"], avg_us=round(v["ms"] * 1e3 / max(1, v["timed"]), 2))
                        for k, v in prof.items()})
    print("RESULT " + json.dumps(rec), flush=True)


if args.child:
    child(args.child)
    sys.exit(0)

what = (f"{args.nx} x {args.ny} slab of 2D Bratu" if args.nz == 0 else
        f"{args.nx} x {args.ny} x {args.nz} slab of 3D heat (G_Euler!)")
print(f"halo self ring: one process, {what}, FD Jv, GMRES(20) restarted, {args.itmax} Arnoldi steps", flush=True)
rows = []
for mode in args.modes.split(","):
    env = dict(os.environ, **ENV[mode])  # (the rigs are operational knobs of the product library)
    env.pop("NK_KBENCH_LIB", None)
    for k in ("NK_HALO_SELF", "NK_HALO_FUSE", "NK_DIST_FORCE", "NK_DIST_MAILBOX", "NK_BLK_INLAUNCH"):
        if k not in ENV[mode]:
            env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", mode, "--nx", str(args.nx), "--ny",
                        str(args.ny), "--nz", str(args.nz), "--itmax", str(args.itmax), "--xdir", args.xdir], env=env,
                       capture_output=True,
                       text=True, timeout=240)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
    if p.returncode != 0 or not lines:
        print(f"mode {mode} failed (rc {p.returncode}):\n{(p.stdout + p.stderr)[-3000:]}", flush=True)
        sys.exit(1)
    r = json.loads(lines[-1][7:])
    rows.append(r)
    print(json.dumps(r), flush=True)
print("\nmode     us/step  jv_fd_dot us  halo_ipc / halo_faces us (launches)  x sha")
for r in rows:
    c = r["classes"]
    jv = c.get("jv_fd_dot", {}).get("avg_us", 0.0)
    h = c.get("halo_ipc") or c.get("halo_faces") or {}
    print(f"{r['mode']:8s} {r['us_per_step']:7.1f}  {jv:11.1f}  {h.get('avg_us', 0.0):8.1f} ({h.get('launches', 0):3d})"
          f"            {r['x_sha']}")
import numpy as np  # noqa: E402

modes = {r["mode"] for r in rows}
if {"blocks", "blocki"} <= modes:
    xb, xk = (np.load(os.path.join(args.xdir, f"x_{m}.npy")) for m in ("blocki", "blocks"))
    print(f"blocki vs blocks: max |dx| / max |x| = {np.max(np.abs(xb - xk)) / np.max(np.abs(xk)):.2e} "
          f"(bitwise: {np.array_equal(xb, xk)})")
if not {"fused", "kernel", "plain", "mbox"} <= modes:
    sys.exit(0)
xf, xk = (np.load(os.path.join(args.xdir, f"x_{m}.npy")) for m in ("fused", "kernel"))
xp, xm = (np.load(os.path.join(args.xdir, f"x_{m}.npy")) for m in ("plain", "mbox"))
print(f"fused vs kernel: max |dx| / max |x| = {np.max(np.abs(xf - xk)) / np.max(np.abs(xk)):.2e} "
      f"(bitwise: {np.array_equal(xf, xk)});  plain vs mbox bitwise: {np.array_equal(xp, xm)}")
