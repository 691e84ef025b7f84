#!/usr/bin/env python3
"""Krylov matvecs/s + achieved HBM GB/s, 2D Bratu 4096^2, GMRES(30) -- BASELINE.json config 2.

One *step* = one inexact-Newton step of newton_krylov_ on the 2D Bratu problem (BASELINE.json
configs[1]): F!(res,u) + ||F|| (fused), one device GMRES(30) solve with the fixed Krylov budget
krylov_kwargs = (restart=true, rtol=0, atol=0, itmax=300) -> 300 Arnoldi matvecs + 9 restart
residual matvecs, the Newton update u -= d, and F! + ||F|| again.  Jv is the north-star fused FD
operator (F(u + eps v) - F(u)) / eps (--jv exact selects the dual-number tangent).

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): weak scaling, every rank owns
a 4096 x 4096 slab of a 4096 x (4096 N) grid; ghost rows go over RCCL send/recv and every inner
product is an RCCL all-reduce.  `value` counts slab matvecs (4096^2-DoF operator applications)
summed over ranks.

Timing: W warm-up steps, barrier + device sync, K timed steps, barrier + device sync; the max over
ranks is reported.  Inputs are resident in HBM before the timed region.  Per-kernel durations come
from HIP events recorded around every launch on the library's stream inside the timed region.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

import _nkpath  # noqa: F401
import ariadne_hip as ah

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
ROOT = os.path.dirname(os.path.abspath(__file__))
# bench kernel class -> rocprofv3 kernel name prefix (for the PMC traffic of profiles/*/pmc_traffic.json)
PMC_NAME = {"mgs_pass": "nk::k_mgs_pass<true,", "mgs_pass_last": "nk::k_mgs_pass<false,",
            "jv_fd_dot_norm": "nk::k_st2d<2, 2, 2,", "jv_exact_dot_norm": "nk::k_st2d<2, 1, 2,",
            "divcopy": "nk::k_divcopy"}
LAMBDA = 3.51382       # examples/bratu.jl:41


def parse():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=4096, help="per-GPU slab is n x n")
    ap.add_argument("--memory", type=int, default=30)
    ap.add_argument("--itmax", type=int, default=300)
    ap.add_argument("--jv", choices=["fd", "exact"], default="fd")
    ap.add_argument("--no-prof", action="store_true", help="do not time kernels with HIP events")
    ap.add_argument("--prof-every", type=int, default=16,
                    help="time every k-th launch of each kernel class (HIP events; k > 1 keeps their cost out)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-itmax", type=int, default=30, help="Arnoldi steps in the CPU-baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: min(16, os.cpu_count())")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r01", "pmc_traffic.json"),
                    help="per-kernel HBM traffic from separate rocprofv3 --pmc passes (tools/pmc_traffic.py)")
    return ap.parse_args()


def slab_ic(nx, ny_loc, ny_glob, y0):
    hx, hy = 1.0 / (nx + 1), 1.0 / (ny_glob + 1)
    xs = np.arange(1, nx + 1) * hx
    ys = np.arange(y0 + 1, y0 + ny_loc + 1) * hy
    return np.ascontiguousarray(np.sin(np.pi * ys)[:, None] * np.sin(np.pi * xs)[None, :]), hx, hy


def cpu_baseline(n, memory, itmax, jv, threads):
    """The C oracle (oracle/nk_oracle.c, test infrastructure) on a bounded sample of the same workload."""
    from oracle import oracle as oc

    oc.set_threads(threads)
    P = oc.bratu2d(n)
    u0 = oc.sin_ic(P)
    F0 = oc.residual(P, u0)
    t0 = time.perf_counter()
    x, st, _ = oc.krylov_solve(P, u0, F0, jv=jv, F0=F0, memory=memory, restart=True, itmax=itmax, atol=0.0, rtol=0.0,
                               history=False)
    dt = time.perf_counter() - t0
    return dict(value=st["n_matvec"] / dt, unit="matvecs/s", cores=oc.get_threads(), kind="port",
                sample=f"oracle/nk_oracle.c GMRES({memory}) restart cycle: {st['n_matvec']} {jv.upper()} matvecs "
                       f"(MGS, same schedule) on the same {n}x{n} Bratu problem, {dt:.2f} s")


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = ah.Context(local)
    ah.set_default_context(ctx)
    if world > 1:
        obj = [ah.dist_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        ctx.init_distributed(rank, world, obj[0])

    n = args.n
    ny_glob = n * world
    u0, hx, hy = slab_ic(n, n, ny_glob, rank * n)
    grid = ah.Grid((n, n), (n, ny_glob), rank * n)
    u = ah.DeviceArray.from_numpy(u0, grid, ctx)
    res = u.zero()
    ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=args.memory))
    p = (hx, hy, LAMBDA)
    kw = dict(restart=True, rtol=0.0, atol=0.0, itmax=args.itmax)

    def step():
        _, r = ah.newton_krylov_(ah.bratu2d_, u, p, res, max_niter=0, tol_rel=0.0, tol_abs=0.0, memory=args.memory,
                                 krylov_kwargs=kw, jv=args.jv, workspace=ws)
        return ws.stats.n_matvec, r

    def barrier():
        ctx.sync()
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    barrier()
    if not args.no_prof:
        ctx.prof_reset()
        ctx.prof_enable(args.prof_every)
    barrier()
    t0 = time.perf_counter()
    matvecs = 0
    last = None
    for _ in range(args.steps):
        mv, last = step()
        matvecs += mv
    ctx.sync()
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    if dist is not None:
        import torch

        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    prof = ctx.prof_read() if not args.no_prof else {}
    ctx.prof_enable(0)

    # algorithmic bytes of every launch (timed launches carry bytes; scale by launches / timed)
    total_bytes = sum(v["bytes"] / max(1, v["timed"]) * v["launches"] for v in prof.values())
    kernels = {k: dict(launches=v["launches"], timed=v["timed"], avg_us=1e3 * v["ms"] / max(1, v["timed"]),
                       gbs=(v["bytes"] / (v["ms"] * 1e-3) / 1e9) if v["ms"] > 0 else None,
                       share=v["ms"] / max(1, v["timed"]) * v["launches"]
                       / max(1e-30, sum(x["ms"] / max(1, x["timed"]) * x["launches"] for x in prof.values())))
               for k, v in sorted(prof.items(), key=lambda kv: -kv[1]["ms"] / max(1, kv[1]["timed"]) * kv[1]["launches"])}

    pmc = {}
    if args.traffic_json and os.path.exists(args.traffic_json):
        with open(args.traffic_json) as f:
            pmc = json.load(f)

    def traffic(name):
        """PMC HBM bytes per launch of this kernel class as a rate over the same launch duration."""
        pre = PMC_NAME.get(name)
        hit = [v for k, v in pmc.items() if pre and k.startswith(pre)]
        return hit[0]["traffic_bytes"] if hit else None

    def roof(name):
        v = prof.get(name)
        if not v or v["ms"] <= 0:
            return None
        ach = v["bytes"] / (v["ms"] * 1e-3) / 1e9
        tb = traffic(name)
        return {"kernel": name, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": round(tb / (v["ms"] / v["timed"] * 1e-3) / 1e9, 1) if tb else None,
                "traffic_bytes_per_launch": tb,
                "traffic_source": os.path.relpath(args.traffic_json, ROOT) if tb else None,
                "bytes_per_launch": v["bytes"] / v["timed"], "avg_us": 1e3 * v["ms"] / v["timed"],
                "timed_launches": v["timed"]}

    dominant = next(iter(kernels), None)
    jv_kernel = "jv_fd_dot_norm" if args.jv == "fd" else "jv_exact_dot_norm"  # Jv fused with V_k = q / h

    if rank == 0:
        value = matvecs * world / elapsed
        out = {
            "metric": "Krylov matvecs/sec + achieved HBM GB/s, 2D Bratu 4096^2",
            "value": round(value, 3),
            "unit": "matvecs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (u0 = sin(pi x) sin(pi y), lambda = 3.51382)",
            "config": {"workload": f"2D Bratu {n}x{n * world} ({n}x{n} per GPU), one inexact-Newton step per step: "
                                   f"GMRES({args.memory}) restart, itmax={args.itmax}, rtol=atol=0, "
                                   f"{args.jv.upper()} Jv",
                       "matvecs_per_step": matvecs // max(1, args.steps), "parallelism": f"slab{world}"},
            "hbm_gbs_algorithmic": round(world * total_bytes / elapsed / 1e9, 1) if total_bytes else None,
            "roofline": roof(dominant) if dominant else None,
            "jv_roofline": roof(jv_kernel),
            "kernels": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                        for k, v in list(kernels.items())[:8]},
            "newton_n_res": last.stats.n_res if last else None,
        }
        if world == 1 and not args.no_cpu_baseline:
            threads = args.cpu_threads or min(16, os.cpu_count() or 1)
            out["cpu_baseline"] = cpu_baseline(n, args.memory, args.cpu_itmax, args.jv, threads)
            out["cpu_baseline"]["value"] = round(out["cpu_baseline"]["value"], 4)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    ws.free()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
