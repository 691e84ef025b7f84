"""GPU tests of the distributed (RCCL) path of libnkhip.so.

* one rank with a forced RCCL communicator: every reduction goes through finalize -> ncclAllReduce
  -> consumer, which must reproduce the single-GPU run bit for bit (same partials, same order);
* 2, 3, 4 and 8 ranks (slabs of a 2D Bratu grid, z-slabs of a 3D heat grid, a periodic ring): halo
  exchange + all-reduced dots against the CPU oracle on the whole grid -- 8 ranks is the decomposition
  of BASELINE configs 4 and 5 (config 4's finite-difference Jv and the Newton solve it drives too);
* the failure path: a rank that stops taking part makes every other rank's next reduction return an
  NK_E_* error in bounded time, and `bench.py --gpus N` then exits non-zero instead of hanging.  Each rank gets its own GPU when the box has enough (then the RCCL
  variants must run: an RCCL error fails the test); on a box with fewer GPUs than ranks they
  share device 0, where only the mailbox transport can run (RCCL refuses -> skip).
"""
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np
import pytest

import _nkpath  # noqa: F401
import ariadne_hip as ah
from oracle import oracle as oc

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def gmres_run(ctx, P, u0, b):
    g = ah.Grid.full(P.nx, P.ny)
    u = ah.DeviceArray.from_numpy(u0, g, ctx)
    bd = ah.DeviceArray.from_numpy(b, g, ctx)
    res = u.zero()
    p = (P.hx, P.hy, P.lam)
    ah.bratu2d_(res, u, p)
    ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=10))
    ah.krylov_solve_(ws, ah.JacobianOperator(ah.bratu2d_, res, u, p), bd, restart=True, atol=0.0, rtol=0.0, itmax=40,
                     history=True)
    return ws.x.to_numpy(), ws.stats, ah.knorm(len(u), u)


def test_forced_rccl_one_rank_is_bitwise(monkeypatch):
    P = oc.bratu2d(48)
    u0 = oc.sin_ic(P)
    b = oc.residual(P, u0)
    plain = ah.Context(0)
    x1, s1, n1 = gmres_run(plain, P, u0, b)
    monkeypatch.setenv("NK_DIST_FORCE", "1")
    forced = ah.Context(0)
    forced.init_distributed(0, 1, ah.dist_unique_id())
    x2, s2, n2 = gmres_run(forced, P, u0, b)
    assert s1.niter == s2.niter == 40
    assert s1.residuals == s2.residuals
    assert np.array_equal(x1, x2) and n1 == n2


def test_forced_one_rank_mailbox_is_bitwise(monkeypatch):
    """The same, with every reduction scalar travelling through the peer mailbox (self-send)."""
    P = oc.bratu2d(48)
    u0 = oc.sin_ic(P)
    b = oc.residual(P, u0)
    plain = ah.Context(0)
    x1, s1, n1 = gmres_run(plain, P, u0, b)
    monkeypatch.setenv("NK_DIST_FORCE", "1")
    monkeypatch.setenv("NK_DIST_MAILBOX", "1")
    forced = ah.Context(0)
    forced.init_distributed(0, 1, ah.dist_unique_id())
    x2, s2, n2 = gmres_run(forced, P, u0, b)
    assert s1.niter == s2.niter == 40
    assert s1.residuals == s2.residuals
    assert np.array_equal(x1, x2) and n1 == n2


def test_mailbox_two_ranks_one_gpu(tmp_path):
    """Two processes on one GPU reduce through each other's mailboxes (IPC, no RCCL)."""
    out = str(tmp_path / "mb")
    rc, log = run_ranks(2, [os.path.join(ROOT, "tests", "mailbox_worker.py"), "--out", out], dict(os.environ))
    assert rc == 0, log[-3000:]
    meta = json.load(open(out + ".json"))
    n = meta["n"]
    y = np.arange(n, dtype=np.float64) % 7
    for k, (dot, nrm2) in enumerate(meta["results"], start=1):
        assert dot == sum((r + k) * y.sum() for r in range(2))
        assert abs(nrm2 - 2 * (y * y).sum()) <= 1e-9 * nrm2  # sqrt then square: a few ulp


_STARTED = set()  # process groups of the ranks this module started


def gpu_holders():
    """Processes of the ranks THIS module started (each in its own session) that still hold the GPU
    open (/dev/kfd): a finished rank's group can linger for a moment while the driver tears its context
    down, and the GPU box allows 16 GPU processes at once.  Unrelated processes on the box are ignored."""
    out = []
    for pid in os.listdir("/proc"):
        if not pid.isdigit():
            continue
        try:
            if os.getpgid(int(pid)) not in _STARTED:
                continue
            if any(os.readlink(f"/proc/{pid}/fd/{fd}") == "/dev/kfd" for fd in os.listdir(f"/proc/{pid}/fd")):
                out.append(int(pid))
        except OSError:
            continue
    return out


def wait_gpu_released(timeout=60.0):
    deadline = time.time() + timeout
    while gpu_holders() and time.time() < deadline:
        time.sleep(0.5)


def run_ranks(world, args, env, timeout=180):
    """Start `world` ranks of a worker script directly (no torch.distributed.run agent: one GPU process
    fewer), after the previous test's ranks have released the GPU; a rank that fails takes the others
    down at once.  Returns (rc, log)."""
    wait_gpu_released()
    port = str(free_port())
    logs = [tempfile.TemporaryFile() for _ in range(world)]
    procs = []
    for r in range(world):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable] + args, env=e, stdout=logs[r], stderr=subprocess.STDOUT,
                                      start_new_session=True))
        _STARTED.add(procs[-1].pid)  # its own session: pgid == pid

    def kill_all():
        for q in procs:
            if q.poll() is None:
                try:
                    os.killpg(q.pid, signal.SIGKILL)
                except OSError:
                    pass
        for q in procs:
            q.wait()

    end, rc = time.time() + timeout, 0
    while any(q.poll() is None for q in procs):
        failed = [q.returncode for q in procs if q.poll() is not None and q.returncode != 0]
        if failed or time.time() > end:
            rc = failed[0] if failed else -9
            kill_all()
            break
        time.sleep(0.2)
    rc = rc or next((q.returncode for q in procs if q.returncode), 0)
    text = []
    for r, f in enumerate(logs):
        f.seek(0)
        text.append(f"--- rank {r} (rc {procs[r].returncode})\n" + f.read().decode(errors="replace")[-4000:])
        f.close()
    if rc == -9 and time.time() > end:
        pytest.fail(f"{world}-rank worker timed out\n" + "\n".join(text)[-3000:])
    return rc, "\n".join(text)


def worker_env(world, **extra):
    """One device per rank when there are enough; else every rank on device 0 (NK_WORKER_SHARED_DEVICE)."""
    env = dict(os.environ, **extra)
    if ah.device_count() < world:
        env["NK_WORKER_SHARED_DEVICE"] = "1"
        # one hardware queue per rank process: 8 ranks x the default 4 would oversubscribe the GPU's
        # queues, which then time-slice -- and every cross-rank reduction waits for a queue to come round
        env["GPU_MAX_HW_QUEUES"] = "1"
    else:
        env.pop("NK_WORKER_SHARED_DEVICE", None)
    return env


def devred_call(fn, meta, ranks, *a, **k):
    """An oracle call in the device's reduction order for the decomposition `ranks` = (px, py, pz) the worker
    ran (its CU count and whether its sweeps ran resident from the worker's path report)."""
    oc.set_devred(True, cus=meta["path"]["resident_blocks"] or 256, ranks=ranks,
                  resident=meta["path"]["sweeps_resident"] > 0)
    try:
        return fn(*a, **k)
    finally:
        oc.set_devred(False)


def check_meta(meta, world):
    if "skip" in meta:
        assert ah.device_count() < world, "RCCL failed although every rank had its own GPU"
        pytest.skip(meta["skip"])


def free_port():
    """A free port BELOW the ephemeral range (Linux: 32768-60999).  A port the kernel hands out for bind(0)
    comes from the range every outgoing connection draws from -- the previous test's gloo / RCCL mesh
    sockets included -- and was taken again before rank 0's store could listen on it (EADDRINUSE, r04)."""
    import random

    rng = random.Random(os.getpid() ^ time.time_ns())
    for _ in range(200):
        port = rng.randrange(20000, 32000)
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", port))
            except OSError:
                continue
            return port
    raise RuntimeError("no free port in 20000-32000")


@pytest.mark.parametrize("transport,world", [("mailbox", 2), ("rccl", 2), ("mailbox", 3), ("rccl", 3), ("mailbox", 4),
                                             ("rccl", 4), ("mailbox", 8), ("rccl", 8), ("host", 2), ("host", 8)])
def test_slabs_match_oracle(tmp_path, world, transport):
    """Slabs of one 2D Bratu grid on `world` ranks: residual, Jv (ghost rows from the neighbours),
    a dot, and a whole Newton-GMRES solve against the oracle on the full grid.  transport=mailbox
    runs ghost planes and reductions through the IPC-mapped peer regions only (no RCCL), so all
    ranks can share the one GPU of the test box; transport=rccl needs one GPU per rank; transport=host
    is the mailbox in host shared memory (NK_DIST_MAILBOX=host: what a launcher that hides the peers'
    devices gets), reductions and (small) ghost planes alike."""
    out = str(tmp_path / "dist")
    env = worker_env(world, **({"NK_DIST_MAILBOX": "host"} if transport == "host" else {}))
    transport = "mailbox" if transport == "host" else transport
    tol = 1e-9  # (8 ranks once needed 1e-6: their spinning reduction consumers starved each other's producers)
    rc, log = run_ranks(world, [os.path.join(ROOT, "tests", "dist_worker.py"), "--out", out, "--transport", transport,
                                "--tol-rel", str(tol)], env)
    assert rc == 0, log[-3000:]
    meta = json.load(open(out + ".json"))
    check_meta(meta, world)
    d = np.load(out + ".npz")
    P = oc.bratu2d(48, 40)
    u0 = oc.sin_ic(P)
    F = oc.residual(P, u0)
    np.testing.assert_array_equal(d["F"], F)  # the shared exp: bit for bit
    np.testing.assert_array_equal(d["jv"], oc.jv_exact(P, u0, d["v"]))  # halo rows came from the neighbours
    np.testing.assert_array_equal(d["jvfd"], oc.jv_fd(P, u0, d["v"], F, eps=1e-7))
    assert abs(meta["dot"] - float(np.sum(u0 * d["v"]))) <= 1e-12 * np.sqrt(u0.size)
    # through the mailbox every rank's sums and their rank-order sum are the device's trees: the oracle in that
    # order gives the Newton solve bit for bit; RCCL's all-reduce has its own order (to the solve's tolerance)
    mb = transport == "mailbox" and meta["path"]["mailbox"]
    if mb:
        oc.set_devred(True, cus=meta["path"]["resident_blocks"] or 256, ranks=(1, world, 1),
                      resident=meta["path"]["sweeps_resident"] > 0)
    try:
        uo, so = oc.newton_krylov(P, u0, memory=10, restart=True, tol_rel=tol)
    finally:
        oc.set_devred(False)
    assert meta["solved"] and so["solved"]
    assert (meta["outer"], meta["inner"]) == (so["outer_iterations"], so["inner_iterations"])
    if mb:
        np.testing.assert_array_equal(d["u"], uo)
    else:
        assert np.max(np.abs(d["u"] - uo)) <= 1e-8 * np.max(np.abs(uo))
    if transport == "mailbox":
        assert meta["path"]["mailbox"] and meta["path"]["mailbox_host"] == (env.get("NK_DIST_MAILBOX") == "host")


@pytest.mark.parametrize("world", [2, 4])
def test_slabs_jacobi_newton_bitwise_in_device_order(tmp_path, world):
    """The preconditioned Newton solve on slabs through the mailbox (N = 1 ./ diag(J) per Newton step, FD Jv):
    every rank's ||N V_k|| from k_diag_apply's scalar chunks over its slab, the ranks' sums in rank order --
    the oracle in the device's order gives counts, and the root, bit for bit."""
    out = str(tmp_path / "dist")
    env = worker_env(world)
    rc, log = run_ranks(world, [os.path.join(ROOT, "tests", "dist_worker.py"), "--out", out, "--transport", "mailbox",
                                "--tol-rel", "1e-8", "--precond", "jacobi", "--jv", "fd", "--nx", "96", "--ny", "80"], env)
    assert rc == 0, log[-3000:]
    meta = json.load(open(out + ".json"))
    d = np.load(out + ".npz")
    assert meta["path"]["mailbox"]
    P = oc.bratu2d(96, 80)
    u0 = oc.sin_ic(P)
    oc.set_devred(True, cus=meta["path"]["resident_blocks"] or 256, ranks=(1, world, 1),
                  resident=meta["path"]["sweeps_resident"] > 0)
    try:
        uo, so = oc.newton_krylov(P, u0, memory=10, restart=True, tol_rel=1e-8, N="jacobi", jv="fd")
    finally:
        oc.set_devred(False)
    assert meta["solved"] and so["solved"]
    assert (meta["outer"], meta["inner"]) == (so["outer_iterations"], so["inner_iterations"])
    np.testing.assert_array_equal(d["u"], uo)


def test_ilu0_pipeline_timeout_recovers_rank_locally(tmp_path):
    """a pipelined ILU(0) sweep that times out on one rank of a distributed solve must recover on
    that rank alone (the apply redone on the level sweep right away) -- a whole-solve redo on one rank would
    pair its reductions with the peers' later ones.  Two ranks on the mailbox, block-Jacobi ILU(0) GMRES(10)
    with a fixed budget, once normally and once with every strip poll allowed a single spin
    (NK_ILU_SPIN_LIMIT=1: the pipelined sweeps time out and the level sweep takes over): the same iterate
    and history bit for bit (both sweeps are bitwise the oracle's), and the timeout really happened."""
    res = {}
    for tag, extra in (("pipe", {}), ("timeout", {"NK_ILU_SPIN_LIMIT": "1"})):
        out = str(tmp_path / tag)
        env = worker_env(2, **extra)
        rc, log = run_ranks(2, [os.path.join(ROOT, "tests", "dist_worker.py"), "--out", out, "--transport", "mailbox",
                                "--nx", "64", "--ny", "512", "--krylov-itmax", "25", "--precond", "ilu0"], env)
        assert rc == 0, log[-3000:]
        res[tag] = (json.load(open(out + ".json")), np.load(out + ".npz"), log)
    assert "pipelined ILU(0) sweep timed out" in res["timeout"][2]
    assert "pipelined ILU(0) sweep timed out" not in res["pipe"][2]
    (m0, d0, _), (m1, d1, _) = res["pipe"], res["timeout"]
    assert m0["niter"] == m1["niter"] == 25
    np.testing.assert_array_equal(d0["h"], d1["h"])
    np.testing.assert_array_equal(d0["x"], d1["x"])


@pytest.mark.parametrize("world,nx,ny,tol", [(2, 48, 40, 1e-9), (4, 64, 96, 1e-9), (8, 48, 40, 1e-9)])
def test_slabs_fd_jv_match_oracle(tmp_path, world, nx, ny, tol):
    """BASELINE config 4's operator on slabs: the finite-difference Jv (the north-star kernel, eps from
    the cross-rank norms of u and v) with its ghost rows from the neighbours, and a Newton-GMRES(10)
    solve driven by it, over the peer mailbox with every rank on the box's GPU.  With a given eps the FD
    quotient is bit-identical to the oracle's (shared exp); with eps from the cross-rank norms, within
    what one ulp of eps does; the Newton count against the oracle's FD solve, the root against the
    oracle's exact-JVP root."""
    out = str(tmp_path / "fd")
    env = worker_env(world)
    rc, log = run_ranks(world, [os.path.join(ROOT, "tests", "dist_worker.py"), "--out", out, "--transport", "mailbox",
                                "--jv", "fd", "--nx", str(nx), "--ny", str(ny), "--tol-rel", str(tol)], env)
    assert rc == 0, log[-3000:]
    meta = json.load(open(out + ".json"))
    d = np.load(out + ".npz")
    P = oc.bratu2d(nx, ny)
    u0 = oc.sin_ic(P)
    F = oc.residual(P, u0)
    np.testing.assert_array_equal(d["F"], F)
    np.testing.assert_array_equal(d["jvfd"], oc.jv_fd(P, u0, d["v"], F, eps=1e-7))  # ghost rows from the neighbours
    ref = oc.jv_fd(P, u0, d["v"], F)
    assert np.max(np.abs(d["jv"] - ref)) <= 1e-7 * np.max(np.abs(ref))  # eps from the cross-rank norms
    exact = oc.jv_exact(P, u0, d["v"])
    assert np.max(np.abs(d["jv"] - exact)) <= 1e-5 * np.max(np.abs(exact))
    _, so = oc.newton_krylov(P, u0, memory=10, restart=True, tol_rel=tol, jv="fd")
    ue, se = oc.newton_krylov(P, u0, memory=10, restart=True, tol_rel=tol)
    assert meta["solved"] and so["solved"] and se["solved"]
    assert meta["outer"] == so["outer_iterations"]
    assert np.max(np.abs(d["u"] - ue)) <= 1e-7 * np.max(np.abs(ue))
    # the FD solve in the device's order (each rank's trees over its slab, ranks summed in rank order): bitwise
    uo, sd = devred_call(oc.newton_krylov, meta, (1, world, 1), P, u0, memory=10, restart=True, tol_rel=tol, jv="fd")
    assert (meta["outer"], meta["inner"]) == (sd["outer_iterations"], sd["inner_iterations"])
    np.testing.assert_array_equal(d["u"], uo)


@pytest.mark.parametrize("transport", ["mailbox", "rccl"])
@pytest.mark.parametrize("world", [2, 3, 8])
def test_periodic_trapezoid_ring_matches_oracle(tmp_path, world, transport):
    """G_Trapezoid! ∘ diffusion! with bc_periodic! on `world` slabs: u_n's ghost planes are exchanged
    as well, and the slabs form a ring (rank 0's lower ghost is rank world-1's last plane; with two
    ranks both neighbours are the same rank).  Residual and exact JVP bit-identical to the oracle on
    the whole grid; one implicit step with equal Newton/Krylov counts."""
    out = str(tmp_path / "ring")
    env = worker_env(world)
    rc, log = run_ranks(world, [os.path.join(ROOT, "tests", "dist_worker.py"), "--out", out, "--transport", transport,
                                "--problem", "heat_periodic"], env)
    assert rc == 0, log[-3000:]
    meta = json.load(open(out + ".json"))
    check_meta(meta, world)
    d = np.load(out + ".npz")
    rng = np.random.default_rng(5)
    un = rng.standard_normal((40, 48))
    u0 = un + 0.01 * rng.standard_normal((40, 48))
    P = oc.heat2d_euler(48, 40, un=un, scheme="trapezoid", bc=oc.BC_PERIODIC)
    assert np.array_equal(d["F"], oc.residual(P, u0))
    assert np.array_equal(d["jv"], oc.jv_exact(P, u0, d["v"]))
    uo, so = oc.newton_krylov(P, u0, tol_abs=6e-6, reorthogonalization=True)
    assert meta["solved"] and so["solved"]
    assert (meta["outer"], meta["inner"]) == (so["outer_iterations"], so["inner_iterations"])
    assert np.max(np.abs(d["u"] - uo)) <= 1e-10
    if transport == "mailbox" and meta["path"]["mailbox"]:  # the ring's reductions in the device's order: bitwise
        ud, _ = devred_call(oc.newton_krylov, meta, (1, world, 1), P, u0, tol_abs=6e-6, reorthogonalization=True)
        np.testing.assert_array_equal(d["u"], ud)


@pytest.mark.parametrize("host", [False, True])
def test_resident_sweep_two_ranks_one_gpu(tmp_path, host):
    """The resident MGS sweep with its per-pass scalars crossing ranks through the peer mailbox: two
    ranks share the test box's GPU, each with a 128-block sweep grid (NK_RES_SHARED: CUs / ranks on
    the GPU) so that both grids are resident together; 1024^2 global (a 1024 x 512 slab per rank: all of q on chip, the
    V_{k+1} hand-over to the next Jv included).  20 restarted GMRES(10) steps against the oracle.
    host: the mailbox in host shared memory -- the resident sweep runs there too."""
    out = str(tmp_path / "dist")
    env = worker_env(2, NK_RES_SHARED="1", **({"NK_DIST_MAILBOX": "host"} if host else {}))
    rc, log = run_ranks(2, [os.path.join(ROOT, "tests", "dist_worker.py"), "--out", out, "--transport", "mailbox",
                            "--nx", "1024", "--ny", "1024", "--krylov-itmax", "20"], env)
    assert rc == 0, log[-3000:]
    meta = json.load(open(out + ".json"))
    d = np.load(out + ".npz")
    P = oc.bratu2d(1024, 1024)
    u0 = oc.sin_ic(P)
    F = oc.residual(P, u0)
    kw = dict(restart=True, atol=0.0, rtol=0.0, itmax=20)
    xo, sto, ho = oc.krylov_solve(P, u0, F, jv="exact", memory=10, **kw)
    assert meta["sweeps"] >= 16  # the resident launches ran (steps 2..10 of both cycles)
    assert meta["path"]["resident_sweep"] and meta["path"]["mailbox_host"] == host
    assert meta["niter"] == sto["niter"] == 20 and meta["n_matvec"] == sto["n_matvec"]
    assert np.allclose(d["h"], ho, rtol=1e-9, atol=0)
    assert np.max(np.abs(d["x"] - xo)) <= 1e-9 * np.max(np.abs(xo))
    # each rank's 128-block sweep tree, the pass scalars added in rank order: bit for bit
    xr, _, hr = devred_call(oc.krylov_solve, meta, (1, 2, 1), P, u0, F, jv="exact", memory=10, **kw)
    np.testing.assert_array_equal(d["h"], hr)
    np.testing.assert_array_equal(d["x"], xr)


def test_eight_ranks_256x256_slabs_fd_gmres(tmp_path):
    """Eight ranks on the box's one GPU at 256 x 256 per rank (a 256 x 2048 grid): the FD operator
    bit for bit, then 40 restarted FD-GMRES(10) steps (eps from the cross-rank norms, every inner
    product through the mailbox) against the oracle on the whole grid in the device's summation order,
    bit for bit -- the size at which the ranks' spinning reduction consumers used to starve each other
    (now one one-block wait per reduction)."""
    out = str(tmp_path / "big")
    world, nx, ny = 8, 256, 2048
    rc, log = run_ranks(world, [os.path.join(ROOT, "tests", "dist_worker.py"), "--out", out, "--transport", "mailbox",
                                "--jv", "fd", "--nx", str(nx), "--ny", str(ny), "--krylov-itmax", "40"], worker_env(world))
    assert rc == 0, log[-3000:]
    meta = json.load(open(out + ".json"))
    d = np.load(out + ".npz")
    P = oc.bratu2d(nx, ny)
    u0 = oc.sin_ic(P)
    F = oc.residual(P, u0)
    np.testing.assert_array_equal(d["F"], F)
    np.testing.assert_array_equal(d["jvfd"], oc.jv_fd(P, u0, d["v"], F, eps=1e-7))
    kw = dict(restart=True, atol=0.0, rtol=0.0, itmax=40)
    # the oracle in the device's summation order (8 slabs of 256 rows, each rank's tree over its slab, the
    # ranks' sums in rank order): the whole history and x bit for bit
    oc.set_devred(True, cus=meta["path"]["resident_blocks"] or 256, ranks=(1, world, 1),
                  resident=meta["path"]["sweeps_resident"] > 0)
    try:
        xo, sto, ho = oc.krylov_solve(P, u0, F, jv="fd", F0=F, memory=10, **kw)
    finally:
        oc.set_devred(False)
    assert meta["niter"] == sto["niter"] == 40 and meta["n_matvec"] == sto["n_matvec"]
    np.testing.assert_array_equal(d["h"], ho)
    np.testing.assert_array_equal(d["x"], xo)


@pytest.mark.parametrize("world,nz", [(2, 24), (3, 24), (8, 24), (2, 64), (3, 72)])
def test_heat3d_midpoint_zslabs_match_oracle(tmp_path, world, nz):
    """3D heat (G_Midpoint!, alpha 0.3) on z-slabs, mailbox transport: the Jv's ghost planes of v travel
    inside the 3D stencil launch (k_st3l's tiles at the slab ends fetch the neighbours' patches).
    Residual, exact and FD JVP bit-identical to the oracle on the whole grid; one implicit step
    with the FD operator: equal Newton / Krylov counts.  nz 64 / 72: two 16-plane z-chunks per slab
    (32 / 24 planes): the lower chunk's tiles fetch the lower ghost plane, the upper chunk's the upper
    one, each from its own inbox in the same launch."""
    out = str(tmp_path / "h3")
    rc, log = run_ranks(world, [os.path.join(ROOT, "tests", "dist_worker.py"), "--out", out, "--transport", "mailbox",
                                "--problem", "heat3d", "--nx", "40", "--ny", "20", "--nz", str(nz)], worker_env(world))
    assert rc == 0, log[-3000:]
    meta = json.load(open(out + ".json"))
    assert meta["mailbox"]
    d = np.load(out + ".npz")
    nx, ny = 40, 20
    rng = np.random.default_rng(9)
    un = rng.standard_normal((nz, ny, nx))
    u0 = un + 0.01 * rng.standard_normal((nz, ny, nx))
    v = rng.standard_normal((nz, ny, nx))
    P = oc.heat3d_euler(nx, ny, nz, un=un, scheme="midpoint", alpha=0.3)
    np.testing.assert_array_equal(d["F"], oc.residual(P, u0))
    np.testing.assert_array_equal(d["jv"], oc.jv_exact(P, u0, v))
    np.testing.assert_array_equal(d["jvfd"], oc.jv_fd(P, u0, v, F0=d["F"], eps=1e-6))
    uo, so = oc.newton_krylov(P, u0, tol_abs=6e-6, jv="fd")
    assert meta["solved"] and so["solved"]
    assert (meta["outer"], meta["inner"]) == (so["outer_iterations"], so["inner_iterations"])
    assert np.max(np.abs(d["u"] - uo)) <= 1e-10
    ud, _ = devred_call(oc.newton_krylov, meta, (1, 1, world), P, u0, tol_abs=6e-6, jv="fd")  # z-slabs: bitwise
    np.testing.assert_array_equal(d["u"], ud)


@pytest.mark.parametrize("fuse_max,form", [(20000, "fused"), (10000, "separate"), (5000, "separate")])
def test_shared_gpu_ghost_plane_form_is_rank_uniform(tmp_path, fuse_max, form):
    """Ranks sharing one GPU carry a Krylov Jv's ghost planes inside the stencil launch only for slabs up
    to kSharedFuseMax points (a big slab's end tiles spin on CUs the peer's producing tiles need: the r05
    30 s/step stall), else through the exchange kernel.  The two forms use different flags, so neighbours
    must agree: the test takes rank-uniform values only -- the most ranks on one GPU and the
    largest slab of an even split from the global spacing.  Two ranks, 3D heat 40 x 20 x 25 split 13 / 12
    planes of 800 points (10400 / 9600), the limit set with NK_SHARED_FUSE_MAX: 10000 lies BETWEEN the two
    local slab sizes (rank-local tests disagreed there and both ranks timed out).  Every rank takes the
    same form: in-launch above both sizes, the exchange kernel otherwise -- and 20 FD-GMRES(20) steps give
    the same bits either way (the form moves no arithmetic)."""
    out = str(tmp_path / "form")
    env = worker_env(2, NK_SHARED_FUSE_MAX=str(fuse_max))
    rc, log = run_ranks(2, [os.path.join(ROOT, "tests", "dist_worker.py"), "--out", out, "--transport", "mailbox",
                            "--problem", "heat3d", "--scheme", "euler", "--nx", "40", "--ny", "20", "--nz", "25",
                            "--krylov-itmax", "20"], env)
    assert rc == 0, log[-3000:]
    meta = json.load(open(out + ".json"))
    assert sorted(meta["planes"]) == [12, 13]
    for q in meta["paths"]:
        assert q["ranks_on_device"] == 2 or ah.device_count() >= 2, q
        assert not q["mailbox_error"], q
        if form == "fused":
            assert q["jv_halo_fused"] > 0 and q["jv_halo_separate"] == 0, q
        else:
            assert q["jv_halo_separate"] > 0 and q["jv_halo_fused"] == 0, q
    d = np.load(out + ".npz")
    ref = str(tmp_path / "ref")
    rc, log = run_ranks(2, [os.path.join(ROOT, "tests", "dist_worker.py"), "--out", ref, "--transport", "mailbox",
                            "--problem", "heat3d", "--scheme", "euler", "--nx", "40", "--ny", "20", "--nz", "25",
                            "--krylov-itmax", "20"], worker_env(2, NK_SHARED_FUSE_MAX=str(1 if form == "fused" else 1 << 30)))
    assert rc == 0, log[-3000:]
    r = np.load(ref + ".npz")
    np.testing.assert_array_equal(d["x"], r["x"])
    np.testing.assert_array_equal(d["h"], r["h"])


@pytest.mark.parametrize("pgrid,nxyz,scheme", [("2,2,2", (40, 20, 24), "midpoint"), ("2,1,1", (40, 20, 24), "midpoint"),
                                                ("1,2,1", (40, 20, 24), "midpoint"), ("1,3,1", (33, 20, 17), "midpoint"),
                                                ("2,2,1", (38, 22, 64), "midpoint"), ("1,2,4", (16, 40, 72), "midpoint"),
                                                ("4,2,1", (130, 18, 20), "midpoint"), ("2,2,2", (48, 40, 36), "euler"),
                                                ("4,2,1", (130, 18, 20), "euler"), ("2,2,2", (40, 20, 24), "trapezoid"),
                                                ("2,2,2", (40, 20, 24), "midpoint-host"),
                                                ("2,2,2", (48, 40, 36), "euler-inlaunch"),
                                                ("1,2,4", (16, 40, 72), "midpoint-inlaunch")])
def test_heat3d_midpoint_blocks_match_oracle(tmp_path, pgrid, nxyz, scheme):
    """BASELINE config 5's decomposition: 3D blocks (px x py x pz process grid, nk_dist_grid) of the 3D
    heat operator (G_Midpoint!, alpha 0.3; G_Euler!, whose Krylov FD Jv recomputes F(u); G_Trapezoid!, whose
    stencil reads u_n's faces too), mailbox transport with every rank on the box's GPU.  Each
    vector's six ghost layers travel in one packed-face launch (k_faces_ipc: z planes into the ghost
    planes, x / y layers into the faces after the trailing plane, which k_st3l reads at the block's x / y
    edges).  Residual, exact and FD JVP bit-identical to the oracle on the whole grid, uneven splits
    included (33 = 11 x 3, 17 planes, 130 = 4 x 32 + 2); one implicit step with the FD operator against the
    oracle in the device's summation order: equal Newton / Krylov counts and u bit for bit, so every inner
    product and Jv of the solve crossed the blocks correctly."""
    world = int(np.prod([int(t) for t in pgrid.split(",")]))
    nx, ny, nz = nxyz
    host = scheme.endswith("-host")  # the mailbox (faces included) in host shared memory
    inl = scheme.endswith("-inlaunch")  # every ghost layer of a Krylov Jv inside its launch (NK_BLK_INLAUNCH=1)
    scheme = scheme.replace("-host", "").replace("-inlaunch", "")
    out = str(tmp_path / "blk")
    env = worker_env(world, **({"NK_DIST_MAILBOX": "host"} if host else {}), **({"NK_BLK_INLAUNCH": "1"} if inl else {}))
    rc, log = run_ranks(world, [os.path.join(ROOT, "tests", "dist_worker.py"), "--out", out, "--transport", "mailbox",
                                "--problem", "heat3d", "--nx", str(nx), "--ny", str(ny), "--nz", str(nz),
                                "--pgrid", pgrid, "--scheme", scheme], env)
    assert rc == 0, log[-3000:]
    meta = json.load(open(out + ".json"))
    assert meta["mailbox"] and meta["path"]["halo_waits"] > 0
    assert meta["path"]["mailbox_host"] == host
    assert (meta["path"]["jv_halo_fused"] > 0) == inl and (meta["path"]["jv_halo_separate"] > 0) == (not inl)
    if scheme == "euler":  # G_Euler!'s FD Jv in the Krylov solve recomputes F(u) -- faces of u included
        assert meta["path"]["jv_fd_f0r"] > 0
    d = np.load(out + ".npz")
    rng = np.random.default_rng(9)
    un = rng.standard_normal((nz, ny, nx))
    u0 = un + 0.01 * rng.standard_normal((nz, ny, nx))
    v = rng.standard_normal((nz, ny, nx))
    P = (oc.heat3d_euler(nx, ny, nz, un=un, scheme="midpoint", alpha=0.3) if scheme == "midpoint"
         else oc.heat3d_euler(nx, ny, nz, un=un, scheme=scheme))
    np.testing.assert_array_equal(d["F"], oc.residual(P, u0))
    np.testing.assert_array_equal(d["jv"], oc.jv_exact(P, u0, v))
    np.testing.assert_array_equal(d["jvfd"], oc.jv_fd(P, u0, v, F0=d["F"], eps=1e-6))
    # the implicit step in the device's summation order (each rank's trees over its block, the ranks' sums
    # in rank order, the Newton driver's norms included): counts and u_{n+1} bit for bit
    oc.set_devred(True, cus=meta["path"]["resident_blocks"] or 256, ranks=tuple(int(t) for t in pgrid.split(",")),
                  resident=meta["path"]["sweeps_resident"] > 0)
    try:
        uo, so = oc.newton_krylov(P, u0, tol_abs=6e-6, jv="fd")
    finally:
        oc.set_devred(False)
    assert meta["solved"] and so["solved"]
    assert (meta["outer"], meta["inner"]) == (so["outer_iterations"], so["inner_iterations"])
    np.testing.assert_array_equal(d["u"], uo)


def test_block_grid_refusals():
    """nk_dist_grid's error behaviour on 2 ranks (1 x 2 x 1): a grid whose size is not the rank count and
    a switch to blocks after a vector exists are NK_E_* errors (the context stays usable), and a
    bc_periodic! residual on blocks is refused (periodic problems keep z-slabs) -- never wrong numbers."""
    import tempfile as _tf

    out = os.path.join(_tf.mkdtemp(), "err")
    rc, log = run_ranks(2, [os.path.join(ROOT, "tests", "dist_worker.py"), "--out", out, "--transport", "mailbox",
                            "--problem", "heat3d", "--nx", "16", "--ny", "12", "--nz", "10", "--pgrid", "1,2,1",
                            "--check-errors"], worker_env(2))
    assert rc == 0, log[-3000:]
    meta = json.load(open(out + ".json"))
    for errs in meta["errors"]:
        assert "px * py * pz must equal the number of ranks" in errs["wrong_grid"], errs
        assert "before allocating vectors" in errs["after_alloc"], errs
        assert "bc_zero! only" in errs["periodic"], errs


@pytest.mark.parametrize("pgrid,nxyz,itmax", [("2,2,2", (128, 96, 80), 40), ("4,2,1", (128, 96, 80), 40),
                                               ("1,1,8", (128, 96, 80), 40), ("2,2,2", (256, 192, 160), 40),
                                               ("2,2,2", (130, 94, 81), 60)])
def test_heat3d_blocks_fd_gmres_budget_matches_oracle(tmp_path, pgrid, nxyz, itmax):
    """8 blocks of a 128 x 96 x 80 grid (64 x 48 x 40 or 32 x 48 x 80 per rank; 1,1,8: z-slabs as the
    control), 256 x 192 x 160 (7.9 M points) and an uneven 130 x 94 x 81: restarted FD-GMRES(20) with a fixed
    budget -- every Jv's six ghost layers and every inner product crossing the blocks -- against the oracle on
    the whole grid, the oracle summing every reduction in the device's order (oracle.set_devred: each rank's
    tree over its own block -- k_st3l's tiles, k_mgs_pass's chunks -- the ranks' sums in rank order as the
    mailbox adds them): F, the whole history and x BIT FOR BIT.  (In the default chunked order the history
    matched only to 1e-8 and had to stop at 30 steps: it plateaus at 1.4957e-5 = 1.4e-8 of its start, the FD
    operator's own accuracy, and when it leaves the plateau depends on the last bits of every sum.)"""
    nx, ny, nz = nxyz
    pg = tuple(int(t) for t in pgrid.split(","))
    world = int(np.prod(pg))
    out = str(tmp_path / "bk")
    rc, log = run_ranks(world, [os.path.join(ROOT, "tests", "dist_worker.py"), "--out", out, "--transport", "mailbox",
                            "--problem", "heat3d", "--nx", str(nx), "--ny", str(ny), "--nz", str(nz), "--pgrid", pgrid,
                            "--krylov-itmax", str(itmax)], worker_env(world))
    assert rc == 0, log[-3000:]
    meta = json.load(open(out + ".json"))
    d = np.load(out + ".npz")
    rng = np.random.default_rng(9)
    un = rng.standard_normal((nz, ny, nx))
    u0 = un + 0.01 * rng.standard_normal((nz, ny, nx))
    P = oc.heat3d_euler(nx, ny, nz, un=un, scheme="midpoint", alpha=0.3)
    F = oc.residual(P, u0)
    np.testing.assert_array_equal(d["F"], F)
    oc.set_devred(True, cus=meta["path"]["resident_blocks"] or 256, ranks=pg,
                  resident=meta["path"]["sweeps_resident"] > 0)
    try:
        xo, sto, ho = oc.krylov_solve(P, u0, F, jv="fd", F0=F, memory=20, restart=True, atol=0.0, rtol=0.0,
                                      itmax=itmax)
    finally:
        oc.set_devred(False)
    assert meta["niter"] == sto["niter"] == itmax and meta["n_matvec"] == sto["n_matvec"]
    assert meta["path"]["halo_waits"] > 0 or world == 1
    np.testing.assert_array_equal(d["h"], ho)
    np.testing.assert_array_equal(d["x"], xo)


@pytest.mark.parametrize("world", [2, 8])
def test_dead_rank_reduction_errors_in_bounded_time(tmp_path, world):
    """A rank that never contributes to a reduction (it stops after the first dot, its context alive):
    every other rank's next kdot must return an NK_E_* error ("a rank's value never arrived") within
    the mailbox spin limit -- never a hang -- and the path report must show the sticky mailbox error."""
    out = str(tmp_path / "fault")
    fault = world - 1
    env = worker_env(world, NK_MB_SPIN_LIMIT=str(1 << 18))
    rc, log = run_ranks(world, [os.path.join(ROOT, "tests", "dist_worker.py"), "--out", out, "--transport", "mailbox",
                                "--fault-rank", str(fault)], env)
    assert rc == 0, log[-3000:]
    meta = json.load(open(out + ".json"))
    P = oc.bratu2d(48, 40)
    v = np.random.default_rng(7).standard_normal((40, 48))
    assert abs(meta["first_dot"] - float(np.sum(oc.sin_ic(P) * v))) <= 1e-12 * np.sqrt(v.size)  # healthy before
    for o in meta["fault"]:
        if o["rank"] == fault:
            assert o["skipped"]
            continue
        assert o["error"] and "never arrived" in o["error"], o
        assert o["seconds"] < 60.0, o
        assert o["path"]["mailbox"] and o["path"]["mailbox_error"], o


def test_dead_rank_block_faces_error_in_bounded_time(tmp_path):
    """3D blocks (2 x 2 x 2): rank 7 stops after the first residual and never pushes its faces again.  The
    next residual (two packed-face exchanges, u and u_n; no reduction) of its three face neighbours (3,
    5, 6) must end in an NK_E_* error within the spin limit, never a hang.  The others exchange only with
    those neighbours or healthy ones: each completes, or -- when a neighbour's second exchange comes only
    after that neighbour's own timeout -- errs in bounded time as well."""
    out = str(tmp_path / "bfault")
    env = worker_env(8, NK_MB_SPIN_LIMIT=str(1 << 18))
    rc, log = run_ranks(8, [os.path.join(ROOT, "tests", "dist_worker.py"), "--out", out, "--transport", "mailbox",
                            "--problem", "heat3d", "--nx", "24", "--ny", "20", "--nz", "16", "--pgrid", "2,2,2",
                            "--fault-rank", "7"], env)
    assert rc == 0, log[-3000:]
    meta = json.load(open(out + ".json"))
    for o in meta["fault"]:
        if o["rank"] == 7:
            assert o["skipped"]
            continue
        assert o["seconds"] < 60.0, o
        if o["rank"] in (3, 5, 6):
            assert o["error"] and "never arrived" in o["error"], o
            assert o["path"]["mailbox_error"], o
        else:
            assert o["error"] is None or "never arrived" in o["error"], o


def test_bench_exits_nonzero_on_a_stuck_rank(tmp_path):
    """`bench.py --gpus 2` whose rank 1 hangs before its first timed step (NK_BENCH_FAULT_RANK=1): rank 0's
    mailbox waits time out into an error, it exits non-zero, the launcher tears the job down -- the bench
    ends with a non-zero status in bounded time instead of hanging."""
    env = worker_env(2, NK_BENCH_FAULT_RANK="1", NK_MB_SPIN_LIMIT=str(1 << 18))
    env.pop("WORLD_SIZE", None)
    wait_gpu_released()
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--transport", "mailbox", "--side", "256",
           "--steps", "2", "--warmup", "1", "--itmax", "30", "--no-cpu-baseline"]
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        log, _ = proc.communicate(timeout=240)
    except subprocess.TimeoutExpired:
        os.killpg(proc.pid, signal.SIGKILL)
        pytest.fail("bench.py hung on a stuck rank")
    text = log.decode(errors="replace")
    assert proc.returncode != 0, text[-3000:]
    assert "never arrived" in text, text[-3000:]


def test_bench_reports_every_ranks_path(tmp_path):
    """The N > 1 bench line carries one path record per rank (transport, resident sweep, in-launch ghost
    planes, launch counts): 8 ranks rehearsed on the box's GPU(s) with the mailbox transport."""
    world = 8
    env = worker_env(world)
    env.pop("WORLD_SIZE", None)
    wait_gpu_released()
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--transport", "mailbox",
           "--side", "256", "--steps", "2", "--warmup", "1", "--itmax", "30", "--no-cpu-baseline"]
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, start_new_session=True)
    try:
        out, err = proc.communicate(timeout=240)
    except subprocess.TimeoutExpired:
        os.killpg(proc.pid, signal.SIGKILL)
        pytest.fail("8-rank bench rehearsal timed out")
    assert proc.returncode == 0, err.decode()[-3000:]
    line = json.loads([ln for ln in out.decode().splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == world and len(line["ranks"]) == world
    assert sorted(r["rank"] for r in line["ranks"]) == list(range(world))
    for r in line["ranks"]:
        assert r["mailbox"] and r["nranks"] == world and not r["mailbox_error"]
        assert r["halo_in_launch"]
        assert r["launches"]["halo_rccl"] == 0 and r["launches"]["allreduce"] == 0
    assert line["config"]["path"]["mailbox_all_ranks"]


def test_self_block_exchange_forms_are_bitwise():
    """3D blocks on one GPU (NK_HALO_SELF=2 rig: the lone rank is its own neighbour on all six sides): a
    restarted FD-GMRES solve with every ghost layer of v exchanged INSIDE the Jv launch (NK_BLK_INLAUNCH=1,
    blk_tile_exchange: exchanging tiles first, patches through the tile flags) gives bit for bit the solution
    of the separate k_faces_ipc launch (the default) -- the layers hold the same values and the partials stay
    tile-indexed -- and the path report says which form ran."""
    wait_gpu_released()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "halo_self.py"), "--nx", "200", "--ny", "72",
                        "--nz", "40", "--itmax", "25", "--modes", "blocks,blocki"], capture_output=True, text=True,
                       timeout=240, env=dict(os.environ))
    assert p.returncode == 0, (p.stdout + p.stderr)[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("blocki vs blocks")][-1]
    assert "(bitwise: True)" in line, p.stdout[-3000:]
    rec = {r["mode"]: r for r in (json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith('{"mode"'))}
    assert rec["blocki"]["path"]["jv_halo_fused"] > 0 and rec["blocki"]["path"]["jv_halo_separate"] == 0
    assert rec["blocks"]["path"]["jv_halo_separate"] > 0 and rec["blocks"]["path"]["jv_halo_fused"] == 0
    assert "halo_faces" in rec["blocks"]["classes"]
    assert rec["blocki"]["classes"].get("halo_faces", {}).get("launches", 0) <= 2  # u's layers only (once per solve)


@pytest.mark.parametrize("dims", [("64", "48", "40"), ("96", "70", "0")])
def test_self_ring_exchange_forms_are_bitwise(dims):
    """One process, a forced one-rank mailbox whose rank is its own lower and upper neighbour (kernel-variant
    build, NK_HALO_SELF): a restarted FD-GMRES solve with the ghost planes (3D) / rows (2D) inside the Jv
    launch gives bit for bit the solution of the separate exchange kernel -- the slab-end-first dispatch of
    the in-launch form changes no sum (stencil partials are indexed by tile) -- and the one-rank mailbox
    without exchange reproduces the plain context."""
    nx, ny, nz = dims
    wait_gpu_released()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "halo_self.py"), "--nx", nx, "--ny", ny, "--nz", nz,
                        "--itmax", "25", "--modes", "plain,mbox,fused,kernel"], capture_output=True, text=True,
                       timeout=240, env=dict(os.environ))
    assert p.returncode == 0, (p.stdout + p.stderr)[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("fused vs kernel")][-1]
    assert "(bitwise: True)" in line and "plain vs mbox bitwise: True" in line, p.stdout[-3000:]
    fused = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith('{"mode": "fused"')][-1]
    assert "halo_ipc" not in fused["classes"] or fused["classes"]["halo_ipc"]["launches"] <= 1  # v's planes in-launch
