"""GPU tests of the resident MGS sweep (launch_mgs_sweep / k_mgs_res in nk_kernels.hip).

From 512^2 up, every Arnoldi step's MGS sweep runs as ONE launch with q held in registers and LDS
(one block per CU, partial sums handed between passes as tagged granules).  These solves cover
its geometries against the CPU oracle -- LDS-only residency (1000^2, whose last 256-wide slot is
partial), LDS + streamed remainder (2560^2), registers + LDS + a partial streamed remainder
(2900 x 2901) -- with and without reorthogonalisation (2k passes per launch; at 1024^2 also with
V_{k+1} handed to the next Jv), run-to-run
determinism, and the in-kernel peer-mailbox reduction (one rank, self-send) bit for bit against
the local one; a heat time step whose sweeps are only partly resident (6144^2); and the optional
fused FD Jv phase (NK_RES_JV=1, a child process).  The full
residency of config 2 (4096^2) is covered by test_hip.py's
test_bratu2d_4096_full_size and by bench.py's CPU/GPU agreement check.
"""
import numpy as np
import pytest

import _nkpath  # noqa: F401
import ariadne_hip as ah
from oracle import oracle as oc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = ah.Context(0)
    ah.set_default_context(c)
    yield c
    c.sync()


def sweeps(ctx, name="mgs_sweep"):
    """Launches of the resident sweep since profiling was enabled: launch_mgs_sweep silently falls back
    to one launch per pass when it cannot keep q on chip, so every test here checks that it ran."""
    return ctx.prof_read().get(name, {}).get("launches", 0)


def solve(P, u, b, ctx=None, **kw):
    ctx = ctx or ah.default_context()
    ctx.prof_reset()
    ctx.prof_enable(1 << 20)  # count launches (time almost none)
    g = ah.Grid.full(P.nx, P.ny)
    ud = ah.DeviceArray.from_numpy(u, g, ctx)
    bd = ah.DeviceArray.from_numpy(b, g, ctx)
    res = ud.zero()
    p = (P.hx, P.hy, P.lam)
    ah.bratu2d_(res, ud, p)
    memory = kw.pop("memory", 10)
    ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=memory))
    ah.krylov_solve_(ws, ah.JacobianOperator(ah.bratu2d_, res, ud, p, jv="exact"), bd, history=True, **kw)
    n_sweeps = sweeps(ctx)
    ctx.prof_enable(0)
    assert n_sweeps > 0, "the resident MGS sweep did not run"
    return ws.x.to_numpy(), ws.stats


@pytest.mark.parametrize("nx,ny,reorth", [(1000, 1000, False), (2560, 2560, False), (2900, 2901, False),
                                          (2900, 2901, True), (1024, 1024, True)])
def test_resident_sweep_matches_oracle(ctx, nx, ny, reorth):
    P = oc.bratu2d(nx, ny)
    u = oc.sin_ic(P)
    b = oc.residual(P, u)
    kw = dict(restart=True, reorthogonalization=reorth, atol=0.0, rtol=0.0, itmax=24)
    x, st = solve(P, u, b, memory=10, **kw)
    cus = ctx.path_info()["resident_blocks"] or 256
    xo, sto, ho = oc.krylov_solve(P, u, b, jv="exact", memory=10, **kw)
    assert st.niter == sto["niter"] == 24 and st.n_matvec == sto["n_matvec"]
    # the same MGS arithmetic per element; only the order of the partial sums differs
    assert np.allclose(np.array(st.residuals), ho, rtol=1e-9, atol=0)
    assert np.max(np.abs(x - xo)) <= 1e-9 * np.max(np.abs(xo))
    # and in the sweep's own order (slot partition over the CUs, the polling wave): bit for bit
    oc.set_devred(True, cus=cus)
    try:
        xr, _, hr = oc.krylov_solve(P, u, b, jv="exact", memory=10, **kw)
    finally:
        oc.set_devred(False)
    np.testing.assert_array_equal(np.array(st.residuals), hr)
    np.testing.assert_array_equal(x, xr)


def test_resident_sweep_deterministic(ctx):
    P = oc.bratu2d(2900, 2901)
    u = oc.sin_ic(P)
    b = oc.residual(P, u)
    runs = [solve(P, u, b, restart=True, atol=0.0, rtol=0.0, itmax=12) for _ in range(2)]
    assert np.array_equal(runs[0][0], runs[1][0])
    assert runs[0][1].residuals == runs[1][1].residuals


@pytest.mark.parametrize("nx,ny", [(1024, 1024), (4096, 6144)])
def test_resident_sweep_mailbox_one_rank_is_bitwise(ctx, monkeypatch, nx, ny):
    """The sweep's per-pass scalars through the peer mailbox (self-send) equal the local ones bit for
    bit -- all of q on chip (1024^2) and two thirds of it (4096 x 6144, config 4's per-rank regime)."""
    P = oc.bratu2d(nx, ny)
    u = oc.sin_ic(P)
    b = oc.residual(P, u)
    plain = ah.Context(0)
    ah.set_default_context(plain)
    x1, s1 = solve(P, u, b, ctx=plain, restart=True, atol=0.0, rtol=0.0, itmax=15)
    monkeypatch.setenv("NK_DIST_FORCE", "1")
    monkeypatch.setenv("NK_DIST_MAILBOX", "1")
    forced = ah.Context(0)
    forced.init_distributed(0, 1, ah.dist_unique_id())
    assert forced.mailbox_active
    ah.set_default_context(forced)
    x2, s2 = solve(P, u, b, ctx=forced, restart=True, atol=0.0, rtol=0.0, itmax=15)
    ah.set_default_context(ctx)
    assert s1.niter == s2.niter == 15
    assert s1.residuals == s2.residuals
    assert np.array_equal(x1, x2)


_JV_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import _nkpath  # noqa: F401
import ariadne_hip as ah
from oracle import oracle as oc
P = oc.bratu2d(1024)
u = oc.sin_ic(P)
b = oc.residual(P, u)
g = ah.Grid.full(P.nx, P.ny)
ud, bd = ah.DeviceArray.from_numpy(u, g), ah.DeviceArray.from_numpy(b, g)
res = ud.zero()
p = (P.hx, P.hy, P.lam)
ah.bratu2d_(res, ud, p)
ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=10))
ctx = ah.default_context()
ctx.prof_enable(1 << 20)
ah.krylov_solve_(ws, ah.JacobianOperator(ah.bratu2d_, res, ud, p, jv="fd"), bd, restart=True, atol=0.0, rtol=0.0,
                 itmax=20, history=True)
steps = ctx.prof_read().get("arnoldi_step", {}).get("launches", 0)  # the fused Jv + sweep launches
np.savez(sys.argv[2], x=ws.x.to_numpy(), h=np.array(ws.stats.residuals), F0=res.to_numpy(), nm=ws.stats.n_matvec,
         steps=steps)
"""


def test_fused_jv_sweep_matches_oracle(tmp_path):
    """NK_RES_JV=1 (the kernel-variant bench build only; not shipped): the FD Jv computed inside the
    resident launch, against the oracle."""
    import os
    import subprocess
    import sys

    out = tmp_path / "jv.npz"
    env = dict(os.environ, NK_RES_JV="1", NK_KBENCH_LIB="1")  # a variant of the kbench build only
    tests = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, "-c", _JV_CHILD, tests, str(out)], env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    d = np.load(out)
    P = oc.bratu2d(1024)
    u = oc.sin_ic(P)
    b = oc.residual(P, u)
    kw = dict(restart=True, atol=0.0, rtol=0.0, itmax=20)
    xo, sto, ho = oc.krylov_solve(P, u, b, jv="fd", F0=d["F0"], memory=10, **kw)
    assert int(d["nm"]) == sto["n_matvec"]
    assert int(d["steps"]) > 0, "the fused Jv + resident sweep launch did not run"
    assert np.allclose(d["h"], ho, rtol=1e-8)
    assert np.max(np.abs(d["x"] - xo)) <= 1e-8 * np.max(np.abs(xo))


def test_heat2d_step_partly_resident_matches_oracle(ctx):
    """One implicit-Euler heat step at 6144^2 (noisy IC): ~44 % of q resident, the rest streamed
    through the same launch; Newton/Krylov counts and the new u equal the oracle's."""
    ah.set_default_context(ctx)
    N = 6144
    rng = np.random.default_rng(0)
    P = oc.heat2d_euler(N)
    u0 = oc.sin_ic(P) + 0.1 * rng.uniform(-1, 1, (N, N))
    un = ah.DeviceArray.from_numpy(u0)
    results = []
    ctx.prof_reset()
    ctx.prof_enable(1 << 20)
    ah.solve(ah.G_Euler_, ah.diffusion_, un, (P.a, P.hx, P.hy, ah.bc_zero_), P.dt, [0.0, P.dt], stats_out=results)
    assert sweeps(ctx) > 0, "the partly resident sweep did not run"
    ctx.prof_enable(0)
    Q = oc.heat2d_euler(N, un=u0)
    ref, so = oc.newton_krylov(Q, u0.copy(), tol_abs=6e-6)
    r = results[0]
    assert r.solved and so["solved"]
    assert (r.stats.outer_iterations, r.stats.inner_iterations) == (so["outer_iterations"], so["inner_iterations"])
    assert np.max(np.abs(un.to_numpy() - ref)) <= 1e-10
    oc.set_devred(True, cus=ctx.path_info()["resident_blocks"] or 256)  # the partly resident sweep's tree
    try:
        ref_dev, _ = oc.newton_krylov(Q, u0.copy(), tol_abs=6e-6)
    finally:
        oc.set_devred(False)
    np.testing.assert_array_equal(un.to_numpy(), ref_dev)


def test_closing_a_context_keeps_another_ones_mailbox(monkeypatch):
    """The mailbox binding is per process and device: closing a context without a mailbox must not
    unbind a live one (it used to, and every later reduction of the live context summed 0 ranks)."""
    P = oc.bratu2d(64)
    u0 = oc.sin_ic(P)
    ref = float(np.linalg.norm(oc.residual(P, u0)))
    monkeypatch.setenv("NK_DIST_FORCE", "1")
    monkeypatch.setenv("NK_DIST_MAILBOX", "1")
    forced = ah.Context(0)
    forced.init_distributed(0, 1, ah.dist_unique_id())
    assert forced.mailbox_active
    monkeypatch.delenv("NK_DIST_FORCE")
    monkeypatch.delenv("NK_DIST_MAILBOX")
    other = ah.Context(0)
    other.close()
    u = ah.DeviceArray.from_numpy(u0, None, forced)
    res = u.zero()
    from ariadne_hip import problems as pr
    n = pr.bratu2d_.residual_norm(res, u, (P.hx, P.hy, P.lam))
    assert abs(n - ref) <= 1e-12 * ref


@pytest.mark.parametrize("jv,reorth,orth_tol,res_tol", [("exact", False, 1e-12, 1e-12), ("fd", False, 1e-9, 1e-9),
                                                       ("exact", True, 1e-14, 1e-12)])
def test_full_size_cycle_properties(ctx, jv, reorth, orth_tol, res_tol):
    """Size-independent properties of two full GMRES(30) cycles at BASELINE config 2's 4096^2 (60
    Arnoldi steps, every MGS sweep resident -- the oracle comparison at this size covers 12): the
    last cycle's basis V_1..V_30 is orthonormal (measured 1.4e-14 exact, 5e-11 FD, 7e-16 with
    reorthogonalization: tools/ortho_probe.py), and the GMRES residual estimate |zeta| equals the
    true ||b - J x|| (7e-16 / 1e-11 relative)."""
    n = 4096
    h = 1.0 / (n + 1)
    xs = np.arange(1, n + 1) * h
    u = ah.DeviceArray.from_numpy(np.sin(np.pi * xs)[:, None] * np.sin(np.pi * xs)[None, :])
    res = u.zero()
    p = (h, h, 3.51382)
    ah.bratu2d_(res, u, p)
    J = ah.JacobianOperator(ah.bratu2d_, res, u, p, jv=jv)
    ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=30))
    ctx.prof_reset()
    ctx.prof_enable(1)
    ah.krylov_solve_(ws, J, res, restart=True, itmax=60, atol=0.0, rtol=0.0, history=True, reorthogonalization=reorth)
    prof = ctx.prof_read()
    ctx.prof_enable(0)
    assert ws.stats.niter == 60 and prof.get("mgs_sweep", {}).get("launches", 0) >= 58
    N = len(u)
    V = [ws.basis(i) for i in range(30)]
    G = np.array([[ah.kdot(N, V[i], V[j]) for j in range(i + 1)] + [0.0] * (29 - i) for i in range(30)])
    G = G + np.tril(G, -1).T
    assert np.max(np.abs(G - np.eye(30))) <= orth_tol
    Jx = u.zero()
    ah.mul_(Jx, J, ws.x)
    r = res.copy()
    ah.kaxpy_(N, -1.0, Jx, r)
    est = ws.stats.residuals[-1]
    assert abs(ah.knorm(N, r) - est) <= res_tol * est
    ws.free()


@pytest.mark.parametrize("case", ["bratu_16384x2048", "heat_8192"])
def test_partly_resident_cycle_properties(ctx, case):
    """The same properties where only part of q fits on chip and the rest streams (non-temporal):
    config 4's 16384 x 2048 slab (half resident) and config 3's 8192^2 heat step (a quarter, with
    reorthogonalization as heat_2D.jl:131 runs it) -- a full GMRES(30) cycle for Bratu, 12 Arnoldi
    steps for the well-conditioned heat Jacobian (cond <= 3: 30 steps would reach the rounding floor),
    exact Jv."""
    if case.startswith("bratu"):
        nx, ny = 16384, 2048
        hx, hy = 1.0 / (nx + 1), 1.0 / (ny + 1)
        u0 = np.sin(np.pi * np.arange(1, ny + 1) * hy)[:, None] * np.sin(np.pi * np.arange(1, nx + 1) * hx)[None, :]
        F, p, reorth, k = ah.bratu2d_, (hx, hy, 3.51382), False, 30
    else:
        n = 8192
        P = oc.heat2d_euler(n, un=np.zeros((1, 1)))
        un = np.sin(np.pi * np.arange(1, n + 1) * P.hy)[:, None] * np.sin(np.pi * np.arange(1, n + 1) * P.hx)[None, :]
        un += 0.1 * np.random.default_rng(0).uniform(-1.0, 1.0, un.shape)
        u0 = un + 0.01
        F = ah.heat2d_euler_
        p, reorth, k = (ah.DeviceArray.from_numpy(un), P.dt, None, (P.a, P.hx, P.hy, ah.bc_zero_), 0.0), True, 12
    u = ah.DeviceArray.from_numpy(np.ascontiguousarray(u0))
    res = u.zero()
    F(res, u, p)
    J = ah.JacobianOperator(F, res, u, p, jv="exact")
    ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=30))
    ctx.prof_reset()
    ctx.prof_enable(1)
    ah.krylov_solve_(ws, J, res, restart=True, itmax=k, atol=0.0, rtol=0.0, history=True, reorthogonalization=reorth)
    prof = ctx.prof_read()
    ctx.prof_enable(0)
    assert ws.stats.niter == k and prof.get("mgs_sweep", {}).get("launches", 0) >= k - 2
    N = len(u)
    V = [ws.basis(i) for i in range(k)]
    G = np.array([[ah.kdot(N, V[i], V[j]) for j in range(i + 1)] + [0.0] * (k - 1 - i) for i in range(k)])
    G = G + np.tril(G, -1).T
    assert np.max(np.abs(G - np.eye(k))) <= 1e-12
    Jx = u.zero()
    ah.mul_(Jx, J, ws.x)
    r = res.copy()
    ah.kaxpy_(N, -1.0, Jx, r)
    est = ws.stats.residuals[-1]
    assert abs(ah.knorm(N, r) - est) <= 1e-10 * est
    ws.free()


_FLAVOUR_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import _nkpath  # noqa: F401
import ariadne_hip as ah
from oracle import oracle as oc
nx, ny = 4096, 6144  # 1.5x the register + LDS capacity: a third of q streams
P = oc.bratu2d(nx, ny)
u = oc.sin_ic(P)
ud = ah.DeviceArray.from_numpy(u)
res = ud.zero()
p = (P.hx, P.hy, P.lam)
ah.bratu2d_(res, ud, p)
ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=8))
ctx = ah.default_context()
ctx.prof_enable(1 << 20)
ah.krylov_solve_(ws, ah.JacobianOperator(ah.bratu2d_, res, ud, p, jv="exact"), res, restart=True, atol=0.0, rtol=0.0,
                 itmax=12, history=True, reorthogonalization=True)
sweeps = ctx.prof_read().get("mgs_sweep", {}).get("launches", 0)
np.savez(sys.argv[2], x=ws.x.to_numpy(), h=np.array(ws.stats.residuals), sweeps=sweeps)
"""


def test_sweep_load_flavours_are_bitwise(tmp_path):
    """The partly resident sweep's cache-policy choices change only how loads and stores are issued
    -- the Infinity-Cache room given to the first streamed slots (NK_RES_NTC), the non-temporal
    streamed remainder (NK_RES_NTS), the first batch loaded across the hand-off (NK_RES_PRE) -- never
    the arithmetic or its order: restarted GMRES with reorthogonalisation, bit for bit -- the product
    library against the kernel-variant bench build (lib/libnkhip_kbench.so) with each knob flipped.
    The vectors' start offsets likewise move addresses only: off, or cycling over two
    vectors instead of eight, the same bits."""
    import os
    import subprocess
    import sys

    tests = os.path.dirname(os.path.abspath(__file__))
    runs = {}
    kb = {"NK_KBENCH_LIB": "1"}  # the knobs are read by the kernel-variant bench build only
    for name, extra in [("default", {}), ("kbench", kb), ("ntc0", dict(kb, NK_RES_NTC="0")),
                        ("ntc_all", dict(kb, NK_RES_NTC="100000")), ("nts0", dict(kb, NK_RES_NTS="0")),
                        ("pre0", dict(kb, NK_RES_PRE="0")), ("offsets0", dict(kb, NK_ALLOC_STAGGER="0")),
                        ("offsets2", dict(kb, NK_ALLOC_STAGGER_MOD="2"))]:
        out = tmp_path / f"{name}.npz"
        r = subprocess.run([sys.executable, "-c", _FLAVOUR_CHILD, tests, str(out)], env=dict(os.environ, **extra),
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, (name, r.stderr[-2000:])
        runs[name] = np.load(out)
    ref = runs["default"]
    assert int(ref["sweeps"]) > 0 and len(ref["h"]) == 13  # r0 and the 12 Arnoldi steps
    for name, d in runs.items():
        assert int(d["sweeps"]) == int(ref["sweeps"]), name
        assert np.array_equal(d["h"], ref["h"]), name
        assert np.array_equal(d["x"], ref["x"]), name
