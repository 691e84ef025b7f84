#!/usr/bin/env python3
"""Krylov matvecs/s + achieved HBM GB/s, 2D Bratu 4096^2, GMRES(30) -- BASELINE.json config 2.

(--workload heat2d / heat3d runs BASELINE configs 3 / 5 instead: implicit-Euler time steps of the
2D heat equation at 8192^2 / the 3D heat equation at 512^3, one time step per step; --scheme
midpoint / trapezoid and --bc periodic select the other implicit.jl schemes and bc_periodic!.)

One *step* = one inexact-Newton step of newton_krylov_ on the 2D Bratu problem (BASELINE.json
configs[1]): F!(res,u) + ||F|| (fused), one device GMRES(30) solve with the fixed Krylov budget
krylov_kwargs = (restart=true, rtol=0, atol=0, itmax=300) -> 300 Arnoldi matvecs + 9 restart
residual matvecs, the Newton update u -= d, and F! + ||F|| again.  Jv is the north-star fused FD
operator (F(u + eps v) - F(u)) / eps (--jv exact selects the dual-number tangent).

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): weak scaling, every rank owns
a 4096 x 4096 slab of a 4096 x (4096 N) grid; ghost rows go over RCCL send/recv and every inner
product is an RCCL all-reduce.  `value` counts slab matvecs (4096^2-DoF operator applications)
summed over ranks.  --global-n G instead splits ONE G x G problem into G/N-row slabs (strong
scaling; --gpus 8 --global-n 16384 is BASELINE config 4); `value` then counts global matvecs.

Timing: W warm-up steps, barrier + device sync, K timed steps, barrier + device sync; the max over
ranks is reported.  Inputs are resident in HBM before the timed region.  Per-kernel durations come
from HIP events recorded around every 64th launch of each kernel class on the library's stream
inside the timed region.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

import _nkpath  # noqa: F401
import ariadne_hip as ah

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
ROOT = os.path.dirname(os.path.abspath(__file__))
# bench kernel class -> rocprofv3 kernel name prefix (for the PMC traffic of profiles/*/pmc_traffic_*.json);
# the stencil template is <KIND, MODE, EPI, VEC, PER>: KIND 2 Bratu 2D, 3/5/7 heat 2D Euler/midpoint/trapezoid,
# 4/6/8 heat 3D; MODE 1 exact, 2 FD; EPI 1 sumsq, 2 dot, 4 dot + fused V_k = q / h store
KIND = {("heat2d", "euler"): 3, ("heat3d", "euler"): 4, ("heat2d", "midpoint"): 5, ("heat3d", "midpoint"): 6,
        ("heat2d", "trapezoid"): 7, ("heat3d", "trapezoid"): 8}


def stencil_prefix(workload, scheme="euler"):
    """Fallback when a profile entry names no instantiation: the product's 2D march / 3D z-march (k_st3l)."""
    if workload == "bratu2d":
        return "nk::k_st2d<2, "
    return f"nk::k_st{'2d' if workload == 'heat2d' else '3l'}<{KIND[workload, scheme]}, "


def pmc_name(workload, kernel, scheme="euler"):
    st = stencil_prefix(workload, scheme)
    return {"mgs_pass": "nk::k_mgs_pass<true,", "mgs_pass_last": "nk::k_mgs_pass<false,", "mgs_sweep": "nk::k_mgs_res<",
            "jv_fd_dot_norm": st + "2, 4,", "jv_exact_dot_norm": st + "1, 4,", "jv_fd_dot": st + "2, 2,",
            "residual_norm": st + "0, 1,", "divcopy": "nk::k_divcopy", "update_x": "nk::k_update_x"}.get(kernel)
LAMBDA = 3.51382       # examples/bratu.jl:41


def log(msg):
    """Progress on stderr (the JSON line alone goes to stdout): the phases after the timed region -- copy
    calibration, CPU baseline, agreement -- take tens of seconds and a silent run looks hung."""
    print(f"bench.py: {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--workload", choices=["bratu2d", "heat2d", "heat3d"], default="bratu2d",
                    help="bratu2d: BASELINE config 2 (default); heat2d: config 3 (8192^2 implicit Euler time "
                         "steps); heat3d: config 5 (512^3 implicit Euler time steps)")
    ap.add_argument("--scheme", choices=["euler", "midpoint", "trapezoid"], default="euler",
                    help="heat workloads: G_Euler! / G_Midpoint! (α = 0.5) / G_Trapezoid! (implicit.jl:8-37)")
    ap.add_argument("--bc", choices=["zero", "periodic"], default="zero",
                    help="heat workloads: bc_zero! / bc_periodic! (heat_2D.jl:15-38)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--side", "--n", dest="n", type=int, default=0,
                    help="per-GPU slab side (default 4096 / 8192 / 512 by workload; spell it --side under torchrun, "
                         "whose own parser claims the --n prefix)")
    ap.add_argument("--global-n", type=int, default=0,
                    help="strong scaling: one global N^dim problem in slabs over the GPUs (--gpus 8 --global-n "
                         "16384 is BASELINE config 4; --workload heat3d --gpus 8 --global-n 512 is config 5)")
    ap.add_argument("--slab-of", type=int, default=0,
                    help="with --global-n on ONE GPU: run the slab one rank of a --slab-of-way decomposition owns "
                         "(rank slab_of // 2, ghost planes zero, no exchange) -- the per-GPU compute of configs 4 / 5 "
                         "before an 8-GPU node is available (--global-n 16384 --slab-of 8)")
    ap.add_argument("--block-of", type=int, default=0,
                    help="heat3d with --global-n G: run ONE rank's block of the N-way 3D-block split (--pgrid auto of N; "
                         "BASELINE config 5: 2x2x2 of 256^3 at G = 512) alone on one GPU, through the block path: the "
                         "BLK stencil instances read x / y ghost faces, and one packed six-face exchange per Jv runs "
                         "over a forced one-rank mailbox whose rank is its own neighbour on both sides of every split "
                         "axis (NK_HALO_SELF=2 rig: those axes wrap onto the block itself -- the cost is what is "
                         "measured; --pgrid px,py,pz picks another split)")
    ap.add_argument("--pgrid", default="",
                    help="heat3d --global-n with N > 1 ranks: 3D blocks px,py,pz (nk_dist_grid; 'auto': the most "
                         "cubic factorisation of N -- 2,2,2 at N = 8, BASELINE config 5's 256^3 blocks) instead of "
                         "z-slabs; every vector's six ghost layers travel in one packed-face launch")
    ap.add_argument("--memory", type=int, default=0, help="Krylov memory (default 30 for bratu2d, 20 for heat)")
    ap.add_argument("--itmax", type=int, default=300)
    ap.add_argument("--jv", choices=["fd", "exact"], default="fd")
    ap.add_argument("--reorth", choices=["auto", "on", "off"], default="auto",
                    help="GMRES reorthogonalization; auto = the reference's own run conditions: on for the heat "
                         "workloads (heat_2D.jl:131 solves with reorthogonalization = true), off for Bratu")
    ap.add_argument("--no-prof", action="store_true", help="do not time kernels with HIP events")
    ap.add_argument("--prof-every", type=int, default=0,
                    help="time every k-th launch of each kernel class (HIP events; k > 1 keeps their cost out of "
                         "the timed region); 0 = 64 for bratu2d (~6000 launches per class), 8 for the heat "
                         "workloads (11 matvecs per step)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--transport", choices=["rccl", "mailbox"], default="rccl",
                    help="N > 1: rccl = nk_dist_init (RCCL bootstrap; peer mailbox + IPC ghost planes when available); "
                         "mailbox = IPC handles over gloo, no RCCL (diagnostic: lets ranks share one GPU -- with "
                         "small slabs only (e.g. --side 1024): a rank's spin-waiting reduction consumers must leave "
                         "the other rank's kernels room on the shared GPU)")
    ap.add_argument("--cpu-itmax", type=int, default=300, help="Arnoldi steps in the CPU-baseline sample (300 = one bench step)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the headline CPU sample (0: the fastest count up to the affinity mask, probed); the per-GPU "
                         "share (OMP_NUM_THREADS) is timed beside it and the machine's nproc reported")
    ap.add_argument("--traffic-json", default="",
                    help="per-kernel HBM traffic from separate rocprofv3 --pmc passes (tools/pmc_traffic.py); "
                         "default profiles/<latest round>/pmc_traffic_<workload>_<side>.json when present (a file "
                         "of another size is never applied)")
    ap.add_argument("--launch-probe", type=int, default=-1, help=argparse.SUPPRESS)  # CPU test of the launcher
    return ap.parse_args()


def cpu_thread_probe(affinity, share):
    """Seconds of a short oracle sample (3 x FD Jv + dot + norm on the 4096^2 Bratu grid) per OpenMP thread
    count -- the per-GPU share, then doubling up to the affinity mask, stopping once a count is clearly
    slower than the best (on a GPU box the mask spans the whole machine while other jobs own most of it:
    256 threads took 135 s for a GMRES cycle that 16 do in 1.5 s).  Returns (fastest count, {count: s})."""
    from oracle import oracle as oc

    P = oc.bratu2d(4096)
    u = oc.sin_ic(P)
    v = np.random.default_rng(1).standard_normal(P.shape)
    F0 = oc.residual(P, u)
    counts = sorted({t for t in (share, 8, 16, 32, 64, 128, 256, 512, affinity) if 0 < t <= affinity})
    probe, best = {}, None
    for t in counts:
        oc.set_threads(t)
        oc.jv_fd(P, u, v, F0)  # warm-up (thread pool)
        t0 = time.perf_counter()
        for _ in range(3):
            w = oc.jv_fd(P, u, v, F0)
            oc.dot(w, v)
            oc.norm(w)
        probe[t] = round(time.perf_counter() - t0, 4)
        log(f"cpu thread probe: {t} threads {probe[t]:.3f} s")
        if best is None or probe[t] < probe[best]:
            best = t
        elif probe[t] > 1.5 * probe[best] or probe[t] > 10.0:
            break
    return best, probe


def jv_alone_calibration(W, ctx, reps=20):
    """BASELINE.md's fused FD Jv as defined there (read u, v, F0; write out: 32 B/pt) -- the `mul!` product
    k_st2d<…, EPI_NONE> -- timed after the timed region on the workload's own u, F(u) and a basis vector
    (the Krylov step runs the 40 B/pt form with <V_1, Jv> fused, jv_roofline)."""
    vs = [b for b in (W.ws.basis(i) for i in range(1, 9)) if b is not None] or [W.u]  # v rotates over V_2 ..
    out = W.u.zero()
    n = len(W.u)
    # between launches a read-only pass over 4 other vectors (537 MB, no dirty lines left to write back during
    # the Jv) evicts the previous launch's operands from the 256 MB Infinity Cache: every launch starts cold
    fl = [W.u.zero(), W.u.zero(), W.u.zero(), W.u.zero()]
    J = ah.JacobianOperator(ah.bratu2d_, W.res, W.u, W.p, jv="fd")
    ah.mul_(out, J, vs[0], eps=1e-7)  # warm
    ctx.sync()
    ctx.prof_reset()
    ctx.prof_enable(1)
    for i in range(reps):
        ah.kdot(n, fl[0], fl[1])
        ah.kdot(n, fl[2], fl[3])
        ah.mul_(out, J, vs[i % len(vs)], eps=1e-7)
    ctx.sync()
    d = ctx.prof_read().get("jv_fd", {})
    ctx.prof_enable(0)
    for f in fl + [out]:
        f.free()
    if not d.get("timed"):
        return None
    us = 1e3 * d["ms"] / d["timed"]
    pts = len(W.u)
    ach = 32.0 * pts / (us * 1e-6) / 1e9
    return {"kernel": d.get("kernel"), "avg_us": round(us, 2), "bytes_per_pt": 32, "achieved": round(ach, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "launches": d["timed"],
            "what": "FD Jv alone (read u, v, F0; write out), BASELINE.md's 32 B/pt definition, HIP events, "
                    "after the timed region; v rotating over basis vectors, every launch cold (a read-only pass "
                    "over 537 MB of other vectors between launches)"}


def copy_calibration(device, n=1 << 27, reps=5):
    """Achievable HBM streaming rate on this GPU: a plain copy over two 1 GiB vectors (nkb_copy, one 16-B
    element per thread, non-temporal), run after the timed region (GB/s on 16 B per element).  The copy
    is a timing hook of the kernel-variant bench build (lib/libnkhip_kbench.so): the product library
    carries no timing hooks.  It runs in a short child process that loads only that build, so the two
    copies of the library (same kernels, same device globals) never share a process."""
    from ariadne_hip import _lib

    if not os.path.exists(_lib.KBENCH_LIB):
        return None
    code = (
        "import ctypes as C, sys\n"
        f"kb = C.CDLL({_lib.KBENCH_LIB!r})\n"
        "kb.nk_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]\n"
        "kb.nk_ctx_destroy.argtypes = [C.c_void_p]\n"
        "kb.nkb_copy.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.POINTER(C.c_double)]\n"
        "h = C.c_void_p()\n"
        f"if kb.nk_ctx_create({int(device)}, C.byref(h)) != 0: sys.exit(1)\n"
        "us = C.c_double()\n"
        f"rc = kb.nkb_copy(h, {int(n)}, {int(reps)}, C.byref(us))\n"
        "kb.nk_ctx_destroy(h)\n"
        "print(us.value if rc == 0 else -1.0)\n")
    try:
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180)
        us = float(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 and r.stdout.strip() else -1.0
    except (subprocess.TimeoutExpired, ValueError, IndexError):
        return None
    if us <= 0:
        return None
    return 16.0 * n / (us * 1e-6) / 1e9


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list) -> int:
    """`bench.py --gpus N` run as a plain process (no torch.distributed.run around it): start the N
    ranks here, one process per GPU (LOCAL_RANK = device), with this same argument list, and return
    the launcher's exit status.  Nothing in this parent touches the GPU (the ranks are children, not
    an exec), so the N = 1 path and the driver's own torchrun launch are unchanged."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + list(argv)
    return subprocess.run(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")).returncode


def exchange_cost(p0, p1, steps, elapsed):
    """What the exchange cost this rank over the timed steps, from the device's own peer-wait clocks
    (nk_path_info): ghost-plane waits of the slab-end tiles (or exchange blocks) and cross-rank reduction
    waits (block 0 of every mailbox all-reduce consumer).  The end tiles of one launch wait side by side,
    so a launch's ghost-plane delay is about their MEAN wait; a reduction's is block 0's wait.
    exchange_share = (launches with an in-launch / separate exchange x mean tile wait + reduction waits)
    / elapsed: an upper bound on the time the exchange kept off the critical path (waits can overlap work)."""
    d = {k: p1[k] - p0[k] for k in ("halo_waits", "reduce_waits", "halo_wait_us", "reduce_wait_us",
                                     "jv_halo_fused", "jv_halo_separate")}
    launches = d["jv_halo_fused"] + d["jv_halo_separate"]
    halo_mean = d["halo_wait_us"] / d["halo_waits"] if d["halo_waits"] else 0.0
    red_mean = d["reduce_wait_us"] / d["reduce_waits"] if d["reduce_waits"] else 0.0
    per_step = (launches * halo_mean + d["reduce_wait_us"]) / max(1, steps)
    return {"halo_waits": d["halo_waits"], "halo_wait_us_mean": round(halo_mean, 3),
            "halo_launches": launches, "reduce_waits": d["reduce_waits"], "reduce_wait_us_mean": round(red_mean, 3),
            "exchange_us_per_step": round(per_step, 1),
            "exchange_share": round(per_step * steps * 1e-6 / elapsed, 4) if elapsed > 0 else None}


def config2_reference():
    """The single-GPU config-2 line to compare a slab line's per-DoF rate with: the newest driver record
    (BENCH_rNN.json at the repo root) of the default 2D Bratu 4096^2 bench, in DoF x matvecs / s."""
    import glob

    for f in sorted(glob.glob(os.path.join(ROOT, "BENCH_r*.json")), reverse=True):
        try:
            with open(f) as fh:
                rec = json.load(fh)
        except (OSError, ValueError):
            continue
        line = rec.get("parsed") if isinstance(rec.get("parsed"), dict) else None
        if line is None:  # else the JSON line among the captured output (stderr lines may follow it)
            tail = (rec.get("run") or {}).get("stdout_tail") or ""
            lines = [ln for ln in tail.splitlines() if ln.startswith('{"metric"')]
            try:
                line = json.loads(lines[-1]) if lines else None
            except ValueError:
                line = None
        if not line or "value" not in line:
            continue
        if line.get("n_gpus") == 1 and "4096x4096 (4096x4096 per GPU)" in line.get("config", {}).get("workload", ""):
            return {"value": line["value"] * 4096 ** 2, "source": f"{os.path.basename(f)}: {line['value']} matvecs/s "
                    "x 4096^2 (2D Bratu 4096^2, one GPU)"}
    return None


def scaling_fields(value, dof_per_unit, paths, workload, slab_of, world, global_n, ref=None, block_of=0):
    """The multi-GPU part of the JSON line (a pure function: tests/test_bench_launcher.py checks an 8-rank
    assembly on CPU).  dof_rate: the north star's >= 6x at 8 GPUs as a per-DoF rate -- DoF x matvecs / s of
    this line against the single-GPU config-2 line (a one-rank slab line has no exchange: its ratio is the
    ceiling the exchange can only lower).  ranks: every rank's path report with its exchange cost;
    exchange: the worst rank's share of the timed region spent waiting for peers."""
    out = {}
    if world > 1 or global_n:
        dof = value * dof_per_unit
        if ref is None and workload == "bratu2d":
            ref = config2_reference()
        out["dof_rate"] = {"dof_matvecs_per_s": round(dof, 1),
                           "vs_config2_single_gpu": round(dof / ref["value"], 3) if ref else None,
                           "config2_reference": ref["source"] if ref else None,
                           "exchange": ("none (one rank's slab alone)" if slab_of else
                                        "self faces on one GPU (no xGMI)" if block_of else "included")}
    if world > 1:
        out["ranks"] = paths  # per rank: transport, resident sweep, in-launch ghost planes, launch counts, cost
        ex = [q.get("exchange") or {} for q in paths]
        shares = [e.get("exchange_share") for e in ex if e.get("exchange_share") is not None]
        out["exchange"] = {"max_share": max(shares) if shares else None,
                           "max_halo_wait_us_mean": max((e.get("halo_wait_us_mean", 0.0) for e in ex), default=None),
                           "max_reduce_wait_us_mean": max((e.get("reduce_wait_us_mean", 0.0) for e in ex), default=None),
                           "what": "per rank: device wall-clock peer waits over the timed steps (ranks[].exchange)"}
    return out


def pgrid_of(spec, world):
    """--pgrid: 'px,py,pz' (product = world) or 'auto' (the most cubic factorisation, x fastest)."""
    if spec == "auto":
        best = None
        for px in range(1, world + 1):
            for py in range(1, world // px + 1):
                if world % (px * py):
                    continue
                pz = world // (px * py)
                key = (max(px, py, pz) - min(px, py, pz), -pz, -py)
                if best is None or key < best[0]:
                    best = (key, (px, py, pz))
        return best[1]
    pg = tuple(int(t) for t in spec.split(","))
    if len(pg) != 3 or int(np.prod(pg)) != world:
        raise SystemExit(f"--pgrid {spec}: three factors whose product is the number of ranks ({world})")
    return pg


def noisy(shape_rows, nx, seed_rows):
    """0.1 U(-1, 1) noise whose every row is seeded by its GLOBAL index, so a slab sees the same field."""
    return np.stack([0.1 * np.random.default_rng([0, int(r)]).uniform(-1.0, 1.0, nx) for r in seed_rows]).reshape(
        shape_rows + (nx,))


class Bratu2D:
    """BASELINE config 2: one inexact-Newton step of 2D Bratu with GMRES(30) and a fixed Krylov budget."""

    def __init__(self, args, ctx, rank, world):
        parts = args.slab_of or world
        if args.slab_of:  # one rank's slab of a parts-way decomposition, alone on this GPU
            rank = parts // 2
        if args.global_n:  # strong scaling: one global G x G problem, G / world rows per rank
            G = args.global_n
            if G % parts:
                raise SystemExit(f"--global-n {G} must be divisible by the number of slabs {parts}")
            n, ny_glob, rows = G, G, G // parts
        else:  # weak scaling: an n x n slab per rank
            n = args.n or 4096
            ny_glob, rows = n * world, n
        self.n, self.world, self.rows = n, world, rows
        self.hx, self.hy = 1.0 / (n + 1), 1.0 / (ny_glob + 1)
        xs = np.arange(1, n + 1) * self.hx
        ys = np.arange(rank * rows + 1, rank * rows + rows + 1) * self.hy
        u0 = np.ascontiguousarray(np.sin(np.pi * ys)[:, None] * np.sin(np.pi * xs)[None, :])
        grid = ah.Grid((n, rows), (n, ny_glob), rank * rows)
        self.u0 = u0
        self.u = ah.DeviceArray.from_numpy(u0, grid, ctx)
        self.res = self.u.zero()
        self.ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(self.res, memory=args.memory))
        self.p = (self.hx, self.hy, LAMBDA)
        self.kw = dict(restart=True, rtol=0.0, atol=0.0, itmax=args.itmax, reorthogonalization=args.reorth == "on")
        self.args = args
        self.jv_kernel = "jv_fd_dot_norm" if args.jv == "fd" else "jv_exact_dot_norm"
        self.scaling = "strong" if args.global_n else "weak"
        self.units_per_matvec = 1 if args.global_n else world  # matvecs counted over the whole problem
        # grid points one counted matvec covers: the global grid (strong scaling / one rank's slab of it
        # alone: `value` counts global matvecs), else one rank's slab (weak scaling: slab matvecs)
        self.dof_per_unit = n * ny_glob if args.global_n else n * rows
        slab = (f"; rank {rank}'s slab of the {parts}-way split ALONE on one GPU (ghost planes zero, no exchange): "
                f"value = slab matvecs/s = the global matvec rate {parts} GPUs would reach without exchange cost"
                if args.slab_of else "")
        self.workload = (f"2D Bratu {n}x{ny_glob} ({n}x{rows} per GPU), one inexact-Newton step per step: "
                         f"GMRES({args.memory}) restart, itmax={args.itmax}, rtol=atol=0, {args.jv.upper()} Jv{slab}")
        self.metric = f"Krylov matvecs/sec + achieved HBM GB/s, 2D Bratu {n}^2"
        self.side = f"{n}x{rows}" if rows != n else str(n)

    def step(self):
        _, r = ah.newton_krylov_(ah.bratu2d_, self.u, self.p, self.res, max_niter=0, tol_rel=0.0, tol_abs=0.0,
                                 memory=self.args.memory, krylov_kwargs=self.kw, jv=self.args.jv, workspace=self.ws)
        return r.n_matvec, r

    def cpu_baseline(self, threads):
        """The C oracle (test infrastructure) on the Krylov solve of one bench step of the same problem --
        bounded: one restart cycle is timed first and the sample shortened to about 20 s of CPU work if the
        whole step would take longer (a host whose cores are busy with other work)."""
        from oracle import oracle as oc

        oc.set_threads(threads)
        # the oracle sums in the device's order (oracle.set_devred, the GPU's CU count as its sweep grid), so
        # the agreement below compares the iterates bit for bit; the arithmetic work is the same either way
        oc.set_devred(True, cus=getattr(self, "dev_cus", 0) or 256)
        P = oc.bratu2d(self.n)
        u0 = oc.sin_ic(P)
        F0 = oc.residual(P, u0)

        def solve(itmax):
            t0 = time.perf_counter()
            x, st, _ = oc.krylov_solve(P, u0, F0, jv=self.args.jv, F0=F0, memory=self.args.memory, restart=True,
                                       itmax=itmax, atol=0.0, rtol=0.0, history=False,
                                       reorthogonalization=self.args.reorth == "on")
            return x, st, time.perf_counter() - t0

        m = self.args.memory
        _, st1, dt1 = solve(m)  # one restart cycle: the per-step cost on these cores
        per_step = dt1 / max(1, st1["niter"])
        itmax = self.args.cpu_itmax
        if per_step * itmax > 20.0:
            itmax = max(m, min(itmax, int(20.0 / per_step) // m * m))
        log(f"cpu baseline: {threads} threads, {dt1:.1f} s per restart cycle -> itmax {itmax}")
        x, st, dt = solve(itmax)
        oc.set_devred(False)
        self.x_cpu, self.cpu_itmax = x, itmax
        return dict(value=st["n_matvec"] / dt, unit="matvecs/s", cores=oc.get_threads(), kind="port",
                    sample=f"oracle/nk_oracle.c: the Krylov solve of one bench step -- GMRES({self.args.memory}) with "
                           f"restarts, itmax={itmax}, {st['n_matvec']} {self.args.jv.upper()} matvecs "
                           f"(MGS, same schedule) on the same {self.n}x{self.n} Bratu problem, {dt:.2f} s")

    def agreement(self):
        """The CPU sample's Newton step repeated on the GPU from the same u0: the north-star quantity is
        ||F(u0 - x)||, which must agree to 1e-10 relative; the raw Krylov iterates are reported as well."""
        from oracle import oracle as oc

        u = ah.DeviceArray.from_numpy(self.u0, self.u.grid, self.u.ctx)
        res = u.zero()
        ah.bratu2d_(res, u, self.p)
        J = ah.JacobianOperator(ah.bratu2d_, res, u, self.p, jv=self.args.jv)
        ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=self.args.memory))
        ah.krylov_solve_(ws, J, res, restart=True, itmax=self.cpu_itmax, atol=0.0, rtol=0.0,
                         reorthogonalization=self.args.reorth == "on")
        x = ws.x.to_numpy()
        ah.kaxpy_(len(u), -1.0, ws.x, u)  # u .-= d (src/Ariadne.jl:344)
        ah.bratu2d_(res, u, self.p)
        n_gpu = ah.knorm(len(res), res)
        ws.free()
        P = oc.bratu2d(self.n)
        n_cpu = float(np.linalg.norm(oc.residual(P, self.u0 - self.x_cpu)))
        d = abs(n_gpu - n_cpu) / n_cpu
        dx = float(np.linalg.norm(x - self.x_cpu) / np.linalg.norm(self.x_cpu))
        return {"quantity": f"||F(u0 - x)|| after one Newton step (GMRES({self.args.memory}), "
                            f"{self.cpu_itmax} Arnoldi steps), GPU vs CPU, relative",
                "value": d, "tolerance": 1e-10, "ok": d <= 1e-10, "n_res_gpu": n_gpu, "n_res_cpu": n_cpu,
                "x_rel_diff": dx, "x_bitwise": bool(np.array_equal(x, self.x_cpu)),
                "cpu_reduction_order": "the device's (oracle.set_devred)"}

    def free(self):
        self.ws.free()


class HeatEuler:
    """BASELINE configs 3 / 5: implicit-Euler time steps (examples/implicit.jl `solve`) of the 2D / 3D heat
    equation, noisy IC, unrestarted GMRES (memory 20), tol_abs = 6e-6; one step = one time step.
    --scheme / --bc: the same loop with G_Midpoint! / G_Trapezoid! and bc_periodic!."""

    def __init__(self, args, ctx, rank, world, dim):
        parts = args.slab_of or args.block_of or world
        if args.slab_of:
            rank = parts // 2
        self.pgrid = None
        if args.pgrid and dim == 3 and world > 1:
            if not args.global_n:
                raise SystemExit("--pgrid splits one --global-n problem into blocks")
            self.pgrid = pgrid_of(args.pgrid, world)
        if args.block_of:  # rank 0's block of the most cubic split (no process grid: the rig's one rank)
            self.pgrid = pgrid_of(args.pgrid or "auto", args.block_of)
            rank = 0
        if args.global_n:  # strong scaling: one global G^dim problem, G / world slab planes per rank
            n = args.global_n
            if n % parts and not self.pgrid:
                raise SystemExit(f"--global-n {n} must be divisible by the number of slabs {parts}")
            planes = n // parts
            glob = (n,) * dim
        else:  # weak scaling: an n^dim block per rank
            n = args.n or (8192 if dim == 2 else 512)
            planes = n
            glob = (n,) * (dim - 1) + (n * world,)
        self.n, self.dim, self.args, self.world = n, dim, args, world
        self.a = 0.01
        hs = [1.0 / (m + 1) for m in glob]
        self.hs = hs
        if dim == 2:
            self.dt = hs[0] ** 2 * hs[1] ** 2 / (2.0 * self.a * (hs[0] ** 2 + hs[1] ** 2))  # heat_2D.jl:72
        else:
            self.dt = 1.0 / (2.0 * self.a * sum(1.0 / h ** 2 for h in hs))
        grid = ah.Grid((n,) * (dim - 1) + (planes,), glob, rank * planes)
        sines = [np.sin(np.pi * np.arange(1, n + 1) * hs[0])]
        rows0 = rank * planes
        if self.pgrid:  # 3D blocks: the process grid first (every vector then carries its x / y faces)
            if not args.block_of:  # (--block-of: the NK_HALO_SELF=2 rig gives the lone rank's vectors faces)
                ctx.set_process_grid(*self.pgrid)
            grid = ah.block(glob, rank, self.pgrid)
            (x0, y0, z0), (nxl, nyl, nzl) = grid.origin, grid.shape_xyz
            zs = np.sin(np.pi * np.arange(z0 + 1, z0 + nzl + 1) * hs[2])
            ys = np.sin(np.pi * np.arange(y0 + 1, y0 + nyl + 1) * hs[1])
            base = zs[:, None, None] * ys[None, :, None] * sines[0][None, None, x0:x0 + nxl]
            rows = [z * n + y for z in range(z0, z0 + nzl) for y in range(y0, y0 + nyl)]
            u0 = base + noisy((nzl, nyl), n, rows)[:, :, x0:x0 + nxl]  # the same field as the slabs see
            planes = nzl
        elif dim == 2:
            ys = np.sin(np.pi * np.arange(rows0 + 1, rows0 + planes + 1) * hs[1])
            u0 = ys[:, None] * sines[0][None, :] + noisy((planes,), n, range(rows0, rows0 + planes))
        else:
            ys = np.sin(np.pi * np.arange(1, n + 1) * hs[1])
            zs = np.sin(np.pi * np.arange(rows0 + 1, rows0 + planes + 1) * hs[2])
            base = zs[:, None, None] * ys[None, :, None] * sines[0][None, None, :]
            u0 = base + noisy((planes, n), n, range(rows0 * n, (rows0 + planes) * n))
        self.scaling = "strong" if args.global_n else "weak"
        self.units_per_matvec = 1 if args.global_n else world
        self.dof_per_unit = int(np.prod(glob)) if args.global_n else n ** (dim - 1) * planes
        self.u0 = np.ascontiguousarray(u0)
        self.un = ah.DeviceArray.from_numpy(self.u0, grid, ctx)
        self.u = self.un.copy()
        self.res = self.u.zero()
        self.ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(self.res, memory=args.memory or 20))
        self.reorth = args.reorth != "off"  # heat_2D.jl:131: krylov_kwargs = (; reorthogonalization = true)
        G = {"euler": ah.G_Euler_, "midpoint": ah.G_Midpoint_, "trapezoid": ah.G_Trapezoid_}[args.scheme]
        self.F = G.bind(ah.diffusion_ if dim == 2 else ah.diffusion3d_)
        bc = ah.bc_periodic_ if args.bc == "periodic" else ah.bc_zero_
        fp = (self.a, hs[0], hs[1], bc) if dim == 2 else (self.a, hs[0], hs[1], hs[2], bc)
        self.p = (self.un, self.dt, None, fp, 0.0)
        self.jv_kernel = "jv_fd_dot_norm" if args.jv == "fd" else "jv_exact_dot_norm"
        shape = "x".join(str(m) for m in glob)
        per_gpu = f"{n}^{dim - 1}x{planes} slab per GPU" if args.global_n else f"{n}^{dim} per GPU"
        if self.pgrid:
            per_gpu = ("x".join(str(m) for m in grid.shape_xyz) + " block per GPU, "
                       + "x".join(str(m) for m in self.pgrid) + " blocks")
        sname = {"euler": "implicit Euler", "midpoint": "implicit midpoint", "trapezoid": "implicit trapezoid"}[args.scheme]
        bcname = "" if args.bc == "zero" else ", bc_periodic!"
        slab = (f"; rank {rank}'s slab of the {parts}-way split ALONE on one GPU (ghost planes zero, no exchange)"
                if args.slab_of else "")
        if args.block_of:
            slab = (f"; rank 0's block of the {parts}-way block split ALONE on one GPU, the ghost faces of every split "
                    "axis exchanged every Jv with itself over a forced one-rank mailbox (NK_HALO_SELF=2: those axes "
                    "wrap onto the block; value = the global matvec rate with this exchange form, without xGMI)")
        self.workload = (f"{dim}D heat {sname}{bcname} {shape} ({per_gpu}), one time step per step: "
                         f"newton_krylov! tol_abs=6e-6, GMRES memory {args.memory or 20} (unrestarted, "
                         f"reorthogonalization={'true' if self.reorth else 'false'}), "
                         f"{args.jv.upper()} Jv, IC sin*sin + 0.1 U(-1,1){slab}")
        self.side = str(n) if planes == n else f"{n}x{planes}"
        if self.pgrid:
            self.side = "block" + "x".join(str(m) for m in grid.shape_xyz)
        self.metric = f"Krylov matvecs/sec + achieved HBM GB/s, {dim}D heat {sname}{bcname} {n}^{dim}"

    def step(self):
        _, r = ah.newton_krylov_(self.F, self.u, self.p, self.res, tol_abs=6.0e-6, memory=self.args.memory or 20,
                                 jv=self.args.jv, workspace=self.ws,
                                 krylov_kwargs=dict(reorthogonalization=self.reorth))
        ah.kcopy_(len(self.un), self.un, self.u)  # uₙ .= u  (implicit.jl:75)
        return r.n_matvec, r

    def cpu_baseline(self, threads):
        from oracle import oracle as oc

        oc.set_threads(threads)
        oc.set_devred(True, cus=getattr(self, "dev_cus", 0) or 256)  # the device's summation order (agreement)
        m = self.n  # bounded sample: one time step of the same problem
        bcc = oc.BC_PERIODIC if self.args.bc == "periodic" else oc.BC_ZERO
        P = (oc.heat2d_euler(m, scheme=self.args.scheme, bc=bcc) if self.dim == 2
             else oc.heat3d_euler(m, scheme=self.args.scheme, bc=bcc))
        u0 = oc.sin_ic(P) + 0.1 * np.random.default_rng(0).uniform(-1, 1, P.shape)
        # bounded sample: implicit time steps of the same problem (implicit.jl:54-78's loop, uₙ .= u) until
        # about 10 s of CPU work (at most 8 steps)
        P.un = u0
        u = u0
        steps, newton, matvecs, dt = 0, 0, 0, 0.0
        while steps < 8 and dt < 10.0:
            t0 = time.perf_counter()
            u, st = oc.newton_krylov(P, u, tol_abs=6e-6, memory=self.args.memory or 20, jv=self.args.jv,
                                     reorthogonalization=self.reorth)
            dt += time.perf_counter() - t0
            log(f"cpu baseline: time step {steps + 1}, {dt:.1f} s so far")
            if steps == 0:  # the first time step, for the CPU/GPU agreement check
                self.cpu_step = (u0, u.copy(), st)
            P.un = u
            steps, newton, matvecs = steps + 1, newton + st["outer_iterations"], matvecs + st["n_matvec"]
        oc.set_devred(False)
        return dict(value=matvecs / dt, unit="matvecs/s", cores=oc.get_threads(), kind="port",
                    sample=f"oracle/nk_oracle.c: {steps} {self.args.scheme} time steps (reorthogonalization="
                           f"{self.reorth}; {newton} Newton, {matvecs} matvecs) of the same {self.dim}D heat problem "
                           f"at {m}^{self.dim} (noise from numpy default_rng(0)), {dt:.2f} s")

    def agreement(self):
        """The CPU sample's first time step repeated on the GPU from the same u0 (same seed, same grid):
        a converged implicit step, so the comparable quantity is the new state u_{n+1} itself (its
        ||F|| sits at the solver tolerance, where it is solve noise) -- GPU vs CPU to 1e-10 relative,
        with the Newton / Krylov counts and both final ||F|| reported."""
        u0, u_cpu, st = self.cpu_step
        g = ah.Grid.full(*u0.shape[::-1])
        un = ah.DeviceArray.from_numpy(u0, g, self.un.ctx)
        u = un.copy()
        res = u.zero()
        p = (un,) + tuple(self.p[1:])
        ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=self.args.memory or 20))
        _, r = ah.newton_krylov_(self.F, u, p, res, tol_abs=6.0e-6, memory=self.args.memory or 20,
                                 jv=self.args.jv, workspace=ws, krylov_kwargs=dict(reorthogonalization=self.reorth))
        u_gpu = u.to_numpy()
        ws.free()
        d = float(np.linalg.norm(u_gpu - u_cpu) / np.linalg.norm(u_cpu))
        same = (r.stats.outer_iterations, r.stats.inner_iterations) == (st["outer_iterations"], st["inner_iterations"])
        return {"quantity": f"u after one implicit {self.args.scheme} time step (converged newton_krylov!, "
                            f"tol_abs=6e-6), GPU vs CPU, relative 2-norm",
                "value": d, "tolerance": 1e-10, "ok": bool(d <= 1e-10 and same),
                "u_bitwise": bool(np.array_equal(u_gpu, u_cpu)), "cpu_reduction_order": "the device's (oracle.set_devred)",
                "counts_gpu": [r.stats.outer_iterations, r.stats.inner_iterations],
                "counts_cpu": [st["outer_iterations"], st["inner_iterations"]],
                "n_res_gpu": r.stats.n_res, "n_res_cpu": st["n_res"]}

    def free(self):
        self.ws.free()


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.workload == "bratu2d" and not args.memory:
        args.memory = 30
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.slab_of and (world > 1 or not args.global_n):
        raise SystemExit("--slab-of runs one rank's slab of a --global-n problem on ONE GPU (--gpus 1)")
    if args.block_of:
        if world > 1 or not args.global_n or args.workload != "heat3d" or args.slab_of:
            raise SystemExit("--block-of runs one rank's 3D block of a --global-n heat3d problem on ONE GPU (--gpus 1)")
        # the rig (read by the library at its first use): a forced one-rank mailbox, the rank its own
        # neighbour on all six sides
        os.environ.update(NK_DIST_FORCE="1", NK_DIST_MAILBOX="1", NK_HALO_SELF="2")
        pg = pgrid_of(args.pgrid or "auto", args.block_of)  # both sides of every split axis (bit 0 z, 1 y, 2 x)
        os.environ["NK_HALO_SELF_AXES"] = str((pg[2] > 1) | (pg[1] > 1) << 1 | (pg[0] > 1) << 2)
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)", file=sys.stderr)
        sys.exit(2)
    if args.launch_probe >= 0:  # CPU test of the launcher: report what this rank was given, no GPU work
        # one write per line (text + newline together): the ranks share the pipe, and print()'s
        # separate write of the newline lets another rank's line land in between when unbuffered
        os.write(1, (json.dumps({"rank": rank, "world": world, "local": local, "argv": sys.argv[1:]}) + "\n").encode())
        sys.exit(args.launch_probe if rank == world - 1 else 0)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world)
    # one GPU per rank (LOCAL_RANK); a box with fewer GPUs than ranks shares them (a rehearsal only:
    # RCCL refuses two ranks on one device, so that needs --transport mailbox and small slabs)
    ndev = ah.device_count()
    if ndev < 1:
        raise SystemExit("bench.py: no GPU visible (the HIP path has no CPU fallback)")
    device = int(os.environ.get("NK_BENCH_DEVICE", local % ndev))  # NK_BENCH_DEVICE: diagnostic override
    ctx = ah.Context(device)
    ah.set_default_context(ctx)
    shared = False
    if dist is not None:
        # ranks share a GPU only if two of them hold the same physical device: (host, PCI bus id of the
        # device this rank opened) -- independent of how a launcher spells visibility (ordinals, UUIDs)
        keys = [None] * world
        dist.all_gather_object(keys, (socket.gethostname(), ctx.path_info()["pci_bus_id"]))
        shared = len(set(keys)) < world
    # NK_BENCH_RCCL_FAIL (tests of the fallback below): "1" -- every rank's RCCL bootstrap "fails" before it
    # starts; "rank:K" -- only rank K's local pre-check fails
    fake = os.environ.get("NK_BENCH_RCCL_FAIL", "")
    fake_fail = fake == "1" or (fake.startswith("rank:") and fake[5:] == str(rank))
    if shared and args.transport == "rccl" and not fake:
        raise SystemExit(f"bench.py: {world} ranks on {ndev} GPU(s): RCCL needs one GPU per rank "
                         "(use --transport mailbox with a small --side to rehearse on fewer GPUs)")
    rccl_error = None
    if world > 1 and args.transport == "rccl":
        # ncclCommInitRank is collective: a rank that fails before entering it would leave the others
        # blocked inside it.  So everything that can fail before it -- rank 0's unique id, a rank's local
        # state (NK_BENCH_RCCL_FAIL=rank:K fakes that) -- is voted on over gloo first; only a unanimous
        # vote enters the collective init.  A failure INSIDE the init that not every rank sees can still
        # block the others there -- the launcher's time limit is then what ends the job.
        obj = [None]
        try:
            if fake_fail:
                raise ah.NKError("NK_BENCH_RCCL_FAIL")
            if rank == 0:
                obj = [ah.dist_unique_id()]
        except ah.NKError as e:
            rccl_error = str(e)
        pre = [None] * world
        dist.all_gather_object(pre, rccl_error)
        failed = [(r, e) for r, e in enumerate(pre) if e]
        if not failed:
            dist.broadcast_object_list(obj, src=0)
            try:
                ctx.init_distributed(rank, world, obj[0])
            except ah.NKError as e:  # (an error every rank returns from: each learns below)
                rccl_error = str(e)
            errs = [None] * world
            dist.all_gather_object(errs, rccl_error)
            failed = [(r, e) for r, e in enumerate(errs) if e]
        if failed:
            # the RCCL bootstrap failed somewhere: every rank starts over on a fresh context with the
            # mailbox alone (IPC handles over gloo) -- the line records it (config.transport)
            rccl_error = f"rank {failed[0][0]}: {failed[0][1]}"
            print(f"bench.py: rank {rank}: RCCL bootstrap failed ({rccl_error}); falling back to the peer mailbox over "
                  "gloo", file=sys.stderr, flush=True)
            ctx.close()
            ctx = ah.Context(device)
            ah.set_default_context(ctx)
            args.transport = "mailbox"
    if world > 1 and args.transport == "mailbox":
        handles = [None] * world
        dist.all_gather_object(handles, ctx.mailbox_handle())
        ctx.mailbox_open(rank, world, b"".join(handles))
    elif world == 1 and os.environ.get("NK_DIST_FORCE") == "1":  # diagnostic: a 1-rank RCCL communicator (every reduction
        ctx.init_distributed(0, 1, ah.dist_unique_id())  # pays the all-reduce path on one GPU)

    if args.workload == "bratu2d":
        W = Bratu2D(args, ctx, rank, world)
    else:
        W = HeatEuler(args, ctx, rank, world, 2 if args.workload == "heat2d" else 3)
    step = W.step

    def barrier():
        ctx.sync()  # every kernel of this process runs on the library's stream: this is the device sync
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    barrier()
    if not args.prof_every:
        args.prof_every = 64 if args.workload == "bratu2d" else 8
    if not args.no_prof:
        ctx.prof_reset()
        ctx.prof_enable(args.prof_every)
    # failure-path rehearsal (tests/test_hip_dist.py): this rank stops taking part -- it hangs before its
    # first timed step, as a stuck peer would; the other ranks' mailbox waits must time out into an
    # NK_E_* error and the whole launch exit non-zero instead of hanging
    fault_rank = int(os.environ.get("NK_BENCH_FAULT_RANK", "-1"))
    barrier()
    path0 = ctx.path_info()  # the peer-wait counters before the timed region
    t0 = time.perf_counter()
    matvecs = 0
    last = None
    for _ in range(args.steps):
        if rank == fault_rank and world > 1:
            print(f"bench.py: rank {rank}: NK_BENCH_FAULT_RANK -- hanging instead of stepping", file=sys.stderr,
                  flush=True)
            time.sleep(3600)
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
    # the path every rank actually ran (transport, resident sweep, in-launch ghost planes, sharing) and
    # the launch counts that prove it: a multi-GPU line names its own path
    path = ctx.path_info()
    path["host"] = socket.gethostname()
    path["exchange"] = exchange_cost(path0, path, args.steps, elapsed)
    path["launches"] = {k: prof.get(k, {}).get("launches", 0)
                        for k in ("mgs_sweep", "mgs_pass", "mgs_pass_last", "halo_ipc", "halo_faces", "halo_rccl",
                                  "allreduce")}
    paths = [path]
    if dist is not None:
        paths = [None] * world
        dist.all_gather_object(paths, path)
    if rank == 0:
        log("timed steps done; copy calibration")
    copy_gbs = copy_calibration(device) if rank == 0 else None
    jv_alone = jv_alone_calibration(W, ctx) if (rank == 0 and world == 1 and args.workload == "bratu2d"
                                                  and args.jv == "fd" and not args.no_prof) else None

    # Two byte counts per kernel class (nk_prof_entry): `bytes` = the operand bytes the kernel moves
    # through the memory hierarchy (every load / store it issues, served by L2, the Infinity Cache or
    # HBM -- "L2 egress"), `dram` = the unique-DRAM model (each distinct operand byte once: a vector
    # re-read by the next pass counts once; a lower bound on HBM traffic, since no gfx950 counter
    # separates Infinity-Cache hits from DRAM reads).  Timed launches carry bytes; scale by launches.
    total_bytes = sum(v.get("bytes_all") or v["bytes"] / max(1, v["timed"]) * v["launches"] for v in prof.values())
    total_dram = sum(v.get("dram_all") or v.get("bytes_all") or 0.0 for v in prof.values())

    def dram_ratio(v):
        return (v.get("dram_all") or 0.0) / v["bytes_all"] if v.get("bytes_all") else 1.0

    kernels = {k: dict(launches=v["launches"], timed=v["timed"], avg_us=1e3 * v["ms"] / max(1, v["timed"]),
                       gbs=(v["bytes"] / (v["ms"] * 1e-3) / 1e9) if v["ms"] > 0 else None,
                       dram_gbs=(dram_ratio(v) * v["bytes"] / (v["ms"] * 1e-3) / 1e9) if v["ms"] > 0 else None,
                       share=v["ms"] / max(1, v["timed"]) * v["launches"]
                       / max(1e-30, sum(x["ms"] / max(1, x["timed"]) * x["launches"] for x in prof.values())))
               for k, v in sorted(prof.items(), key=lambda kv: -kv[1]["ms"] / max(1, kv[1]["timed"]) * kv[1]["launches"])}

    pmc = {}
    tag = args.workload + ("" if args.scheme == "euler" else "_" + args.scheme) + ("" if args.bc == "zero" else "_periodic")
    if not args.traffic_json:
        rounds = sorted(d for d in os.listdir(os.path.join(ROOT, "profiles")) if d.startswith("r"))
        for rd in reversed(rounds):  # the newest PMC pass of exactly this workload and size
            f = os.path.join(ROOT, "profiles", rd, f"pmc_traffic_{tag}_{W.side}.json")
            if os.path.exists(f):
                args.traffic_json = f
                break
    if args.traffic_json and os.path.exists(args.traffic_json):
        with open(args.traffic_json) as f:
            pmc = json.load(f)

    def traffic(name):
        """PMC HBM bytes per launch of this kernel class: the entry of exactly the instantiation this run
        launched (nk_prof_entry.kernel, stencil classes), else the class's kernel-name prefix."""
        inst = prof.get(name, {}).get("kernel")
        if inst:
            return pmc[inst]["traffic_bytes"] if inst in pmc else None
        pre = pmc_name(args.workload, name, args.scheme)
        hit = [v for k, v in pmc.items() if pre and k.startswith(pre)]
        return hit[0]["traffic_bytes"] if hit else None

    def roof(name):
        v = prof.get(name)
        if not v or v["ms"] <= 0:
            return None
        ach = v["bytes"] / (v["ms"] * 1e-3) / 1e9
        if ach <= 0:
            return None
        tb = traffic(name)
        # mean algorithmic bytes over ALL launches (a sweep's size varies with the Arnoldi step; the
        # timed launches are every 64th one).  PMC traffic comes from a separate run with the same
        # GMRES(30) cycle structure, so traffic / algorithmic bytes per launch is compared as a ratio.
        bpl = v.get("bytes_all", 0.0) / v["launches"] if v.get("bytes_all") else v["bytes"] / v["timed"]
        dr = dram_ratio(v)
        # avg_us: the mean launch duration over ALL launches at the measured rate (the timed launches
        # of a kernel whose size varies per launch are not a uniform sample of the sizes);
        # avg_us_timed: the plain mean of the timed launches
        return {"kernel": name, "instantiation": v.get("kernel") or None, "bound": "hbm", "achieved": round(ach, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4),
                "bytes_basis": "l2_egress: every operand byte the kernel loads / stores (any cache level; "
                               "PMC FETCH/WRITE_SIZE count the same, Infinity-Cache hits included)",
                "dram_model": {"achieved": round(ach * dr, 1), "frac": round(ach * dr / HBM_PEAK_GBS, 4),
                               "bytes_per_launch": bpl * dr,
                               "basis": "unique operand bytes (re-reads counted once: a lower bound on DRAM traffic)"},
                "traffic": round(ach * tb / bpl, 1) if tb else None,
                "traffic_bytes_per_launch": tb,
                "traffic_source": os.path.relpath(args.traffic_json, ROOT) if tb else None,
                "frac_of_copy": round(ach / copy_gbs, 4) if copy_gbs else None,
                "bytes_per_launch": bpl, "avg_us": round(1e6 * bpl / (ach * 1e9), 3),
                "avg_us_timed": 1e3 * v["ms"] / v["timed"], "timed_launches": v["timed"]}

    # the kernel with the largest share of the time among those that move operand bytes (with ranks sharing
    # one GPU, the one-block cross-rank waits -- k_finalize, no bytes -- can carry the largest share)
    dominant = next((k for k, v in kernels.items() if v["gbs"]), None)
    # the Jv of the Arnoldi steps: fused with V_k = q / h (jv_*_dot_norm), or reading V_k as stored
    # by the previous resident sweep (jv_*_dot) -- whichever carries more of the time
    jv_kernel = max((W.jv_kernel, W.jv_kernel.replace("_dot_norm", "_dot")),
                    key=lambda k: kernels.get(k, {}).get("share", -1.0))

    if rank == 0:
        value = matvecs * getattr(W, "units_per_matvec", world) / elapsed
        out = {
            "metric": W.metric,
            "value": round(value, 3),
            "unit": "matvecs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": getattr(W, "scaling", "weak"),
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (see config.workload)",
            "config": {"workload": W.workload, "matvecs_per_step": matvecs // max(1, args.steps),
                       "parallelism": ((f"block 1 of {args.block_of} (one GPU, self faces)") if args.block_of else
                                       ("blocks" + "x".join(str(m) for m in W.pgrid)) if getattr(W, "pgrid", None)
                                       else (f"slab{world}" if not args.slab_of else f"slab 1 of {args.slab_of} (one GPU)")),
                       "reorthogonalization": bool(getattr(W, "reorth", args.reorth == "on")),
                       "devices": (f"{min(world, ndev)} GPU(s) for {world} rank(s) (shared: rehearsal)" if shared
                                   else f"{world} GPU(s), one per rank"),
                       "transport": (args.transport if world > 1 else "local")
                                    + (f" (RCCL bootstrap failed: {rccl_error})" if rccl_error else ""),
                       "reductions": ("peer mailbox (IPC/xGMI)" if ctx.mailbox_active else
                                      ("ncclAllReduce" if world > 1 else "local")),
                       "path": {"mailbox_all_ranks": all(q["mailbox"] for q in paths),
                                "resident_sweep_all_ranks": all(q["launches"]["mgs_sweep"] > 0 for q in paths),
                                "halo_in_launch_all_ranks": all(q["halo_in_launch"] for q in paths) if world > 1
                                else None,
                                "mailbox_errors": sum(1 for q in paths if q["mailbox_error"])}},
            # whole job: operand bytes through the memory hierarchy, and the unique-DRAM model, per second
            "gbs_l2_egress_wholejob": round(world * total_bytes / elapsed / 1e9, 1) if total_bytes else None,
            "gbs_dram_model_wholejob": round(world * total_dram / elapsed / 1e9, 1) if total_dram else None,
            "roofline": roof(dominant) if dominant else None,
            "jv_roofline": roof(jv_kernel),
            "jv_alone": jv_alone,
            "kernels": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                        for k, v in list(kernels.items())[:8]},
            "newton_n_res": last.stats.n_res if last else None,
            # what plain streaming reaches on this GPU (roofline.frac_of_copy divides by it): the spec
            # 8 TB/s is not reachable by any access pattern (MI355X_MICROARCH.md: 6.29 TB/s best measured)
            "calibration": {"copy_gbs": round(copy_gbs, 1) if copy_gbs else None,
                            "what": "y = x over 2 x 1 GiB (HBM, beyond the Infinity Cache), one 16-B element per "
                                    "thread, non-temporal load + store (the fastest copy of tools/stream_probe.py), "
                                    "mean of 5 launches, after the timed region"},
        }
        out.update(scaling_fields(value, W.dof_per_unit, paths, args.workload, args.slab_of, world, args.global_n,
                                  block_of=args.block_of))
        if args.block_of:
            out["ranks"] = paths  # the rig's path report: faces exchanged, BLK instances, peer waits
        if world == 1 and not args.no_cpu_baseline and not args.global_n:
            # the node's host cores: the fastest thread count the process's affinity mask offers (the
            # headline figure), and the per-GPU share the box gives one GPU (OMP_NUM_THREADS, 16 there)
            # beside it; nproc is the machine's full count
            affinity = len(os.sched_getaffinity(0))
            share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
            probe = {}
            if args.cpu_threads:
                threads = args.cpu_threads
            else:  # the fastest thread count the affinity mask offers (on a shared host, more is not faster)
                threads, probe = cpu_thread_probe(affinity, share)
            log(f"cpu baseline on {threads} threads (affinity mask {affinity}, probe {probe})")
            W.dev_cus = paths[0].get("resident_blocks") or 0  # the sweep grid the oracle's device order follows
            cb = W.cpu_baseline(threads)
            cb["value"] = round(cb["value"], 4)
            cb["host_cpus"] = {"nproc": os.cpu_count(), "affinity": affinity,
                               "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
                               "thread_probe_s": probe,
                               "threads_rule": "the faster of two samples: the per-GPU share (OMP_NUM_THREADS) and "
                                               "the fastest count of a short probe up to the affinity mask (a Bratu "
                                               "4096^2 FD Jv + dot + norm, 3x, per count)"}
            if share and share != threads:
                log(f"cpu baseline on the per-GPU share, {share} threads")
                sh = W.cpu_baseline(share)
                sh["value"] = round(sh["value"], 4)
                if sh["value"] > cb["value"]:  # the headline is the faster of the two measured samples
                    sh["host_cpus"] = cb.pop("host_cpus")
                    cb, sh = sh, cb
                cb["other_sample"] = {"value": sh["value"], "unit": sh["unit"], "cores": sh["cores"],
                                      "sample": sh["sample"]}
            out["cpu_baseline"] = cb
            if hasattr(W, "agreement"):
                log("cpu/gpu agreement")
                out["cpu_gpu_agreement"] = W.agreement()
        else:
            out["cpu_baseline"] = None
        sys.stdout.write(json.dumps(out) + "\n")
        sys.stdout.flush()
    W.free()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
