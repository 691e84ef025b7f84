"""GMRES parity at any length: the oracle in its device-order mode (oracle.set_devred,
nk_oracle.c OC_DEVRED) sums every reduction of a one-rank 2D GMRES solve in exactly the tree the product's
kernels use -- k_st2d's tile partials for <V_1, J V_k> and the restart residual, the resident sweep's slot
partition and polling wave for the MGS passes (k_mgs_pass's chunks where the sweep does not run),
k_sumsq / k_update_x for ||b||, ||u||, ||x||, reduce_input / k_finalize for every consumer.  With the
operator already bit-identical (shared exp, same association order), the whole restarted FD-GMRES
history and the iterate then agree BIT FOR BIT with the device, however many restarts -- instead of
drifting apart by summation order (1e-8 over 15 restarts in the default mode).

Preconditioned solves (Jacobi, ILU(0), the inner-GMRES N; left M; FGMRES; CG) and Newton solves are
compared the same way (the preconditioners' own norms and dots in their kernels' trees).

Tolerance: none (np.array_equal).  Hardware parameter: the sweep grid is the GPU's CU count, read from
the device's own path report and handed to the oracle."""
import os

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


def problem(kind, nx, ny):
    if kind == "bratu":
        P = oc.bratu2d(nx, ny)
        u = oc.sin_ic(P)
        return P, u, ah.bratu2d_, (1.0 / (nx + 1), 1.0 / (ny + 1), P.lam)
    rng = np.random.default_rng(3)
    un = oc.sin_ic(oc.bratu2d(nx, ny)) + 0.1 * rng.standard_normal((ny, nx))
    P = oc.heat2d_euler(nx, ny, un=un)
    u = un + 0.01 * rng.standard_normal((ny, nx))
    return P, u, None, un


def device_solve(ctx, kind, P, u, F_, p, un, memory, itmax, jv, reorth):
    grid = ah.Grid.full(P.nx, P.ny)
    ud = ah.DeviceArray.from_numpy(u, grid, ctx)
    if kind != "bratu":
        und = ah.DeviceArray.from_numpy(un, grid, ctx)
        F_ = ah.G_Euler_.bind(ah.diffusion_)
        p = (und, P.dt, None, (P.a, P.hx, P.hy, ah.bc_zero_), 0.0)
    res = ud.zero()
    F_(res, ud, p)
    ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=memory))
    J = ah.JacobianOperator(F_, res, ud, p, jv=jv)
    ah.krylov_solve_(ws, J, res, restart=True, atol=0.0, rtol=0.0, itmax=itmax, history=True,
                     reorthogonalization=reorth)
    return ws.x.to_numpy(), ws.stats, res.to_numpy(), ctx.path_info()


@pytest.mark.parametrize("kind,nx,ny,memory,itmax,jv,reorth", [
    ("bratu", 1024, 1024, 30, 90, "fd", False),   # 3 restarted GMRES(30) cycles, resident sweep, 128 tiles x 2
    ("bratu", 512, 384, 20, 60, "fd", False),     # uneven slot partition: some sweep blocks own 2 slots, some 1
    ("heat", 1024, 512, 20, 60, "fd", True),      # reorthogonalisation: 2k passes per sweep
    ("bratu", 256, 256, 10, 60, "exact", False),  # below one slot per CU: the k_mgs_pass chain every step
])
def test_restarted_gmres_bitwise_in_device_order(ctx, kind, nx, ny, memory, itmax, jv, reorth):
    P, u, F_, p = problem(kind, nx, ny)
    x, st, F0, path = device_solve(ctx, kind, P, u, F_, p, p, memory, itmax, jv, reorth)
    if kind == "heat":
        np.testing.assert_array_equal(F0, oc.residual(P, u))
    cus = path["resident_blocks"] or 256
    oc.set_devred(True, cus=cus)
    try:
        xo, so, ho = oc.krylov_solve(P, u, F0, jv=jv, F0=F0, memory=memory, restart=True, atol=0.0, rtol=0.0,
                                     itmax=itmax, reorthogonalization=reorth)
    finally:
        oc.set_devred(False)
    assert st.niter == so["niter"] == itmax and st.n_matvec == so["n_matvec"]
    h = np.array(st.residuals)
    np.testing.assert_array_equal(h, ho)
    np.testing.assert_array_equal(x, xo)
    # and the default (chunked) oracle order is NOT the device's: the bits above come from the emulation
    xd, _, hd = oc.krylov_solve(P, u, F0, jv=jv, F0=F0, memory=memory, restart=True, atol=0.0, rtol=0.0,
                                itmax=itmax, reorthogonalization=reorth)
    assert not np.array_equal(hd, h)


@pytest.mark.parametrize("kind,nx,ny,kw", [
    ("bratu", 128, 96, dict(tol_rel=1e-8, memory=20, krylov_kwargs=dict(restart=True))),    # 2785 GMRES steps
    ("bratu", 160, 160, dict(tol_rel=1e-6, memory=30, krylov_kwargs=dict(restart=True))),
    ("heat", 1024, 1024, dict(tol_abs=6e-6, memory=20, krylov_kwargs=dict(reorthogonalization=True))),  # resident
])
def test_newton_bitwise_in_device_order(ctx, kind, nx, ny, kw):
    """Whole inexact-Newton solves (src/Ariadne.jl:288-372, Eisenstat-Walker forcing, FD Jv) against the oracle
    in the device's order, the Newton driver's own norms included (||F(u)|| from the residual kernel's tiles,
    ||u|| from the update fused into the solve's last x update): equal outer / inner counts, the ||F||
    history and the root BIT FOR BIT.  (In the default order a tight tolerance can already move the inner
    count: 3436 against 3434 on a 128 x 96 Bratu solve at tol_rel 1e-10.)  Sizes keep the oracle's CPU side
    within seconds (2D Bratu near its fold needs thousands of GMRES steps per solve)."""
    P, u, F_, p = problem(kind, nx, ny)
    grid = ah.Grid.full(P.nx, P.ny)
    ud = ah.DeviceArray.from_numpy(u, grid, ctx)
    if kind != "bratu":
        und = ah.DeviceArray.from_numpy(p, grid, ctx)
        F_ = ah.G_Euler_.bind(ah.diffusion_)
        p = (und, P.dt, None, (P.a, P.hx, P.hy, ah.bc_zero_), 0.0)
    hist = []
    ud, r = ah.newton_krylov_(F_, ud, p, jv="fd", callback=lambda u_, res_, n: hist.append(n), **kw)
    path = ctx.path_info()
    okw = {k: v for k, v in kw.items() if k != "krylov_kwargs"}
    okw.update(kw.get("krylov_kwargs", {}))
    oc.set_devred(True, cus=path["resident_blocks"] or 256)
    try:
        uo, so = oc.newton_krylov(P, u, jv="fd", **okw)
    finally:
        oc.set_devred(False)
    assert r.solved and so["solved"]
    assert (r.stats.outer_iterations, r.stats.inner_iterations) == (so["outer_iterations"], so["inner_iterations"])
    np.testing.assert_array_equal(np.array(hist), so["n_res_history"])
    np.testing.assert_array_equal(ud.to_numpy(), uo)


def test_config1_newton_cg_bitwise_in_device_order(ctx, golden_dir):
    """BASELINE config 1 (examples/bratu.jl:59-63: 1D Bratu N = 1000, algo = :cg, exact JVP) against the oracle
    in the device's order (k_st1d's 256-point partials, k_sumsq / k_cg_update's chunks): thousands of CG
    iterations on cond(J) ~ 1.75e8, whose counts move by ~9 % under a 1-ulp change of u0 in the default
    order (test_hip.py::test_newton_bratu1d_cg_config1 compares only the outcome there) -- here equal outer /
    inner counts and u bit for bit."""
    g = np.load(os.path.join(golden_dir, "bratu1d_n1000.npz"))
    P = oc.bratu1d(1000)
    u = ah.DeviceArray.from_numpy(g["u0"], None, ctx)
    hist = []
    u, r = ah.newton_krylov_(ah.bratu_, u, (P.hx, P.lam), u.similar(), algo="cg",
                             callback=lambda u_, res_, n: hist.append(n))
    oc.set_devred(True)
    try:
        uo, so = oc.newton_krylov(P, g["u0"], algo="cg")
    finally:
        oc.set_devred(False)
    assert r.solved and so["solved"]
    assert (r.stats.outer_iterations, r.stats.inner_iterations) == (so["outer_iterations"], so["inner_iterations"])
    np.testing.assert_array_equal(np.array(hist), so["n_res_history"])
    np.testing.assert_array_equal(u.to_numpy(), uo)
    assert np.max(np.abs(uo - g["true_sol"])) < 3e-4


# ----------------------------------------------------------------------------- preconditioned solves
def _prec(kind, J, P, u0):
    """The device preconditioner for J(u0) and the oracle's form of the same operator."""
    if kind == "jacobi":
        return ah.jacobi(J), ("diag", oc.jacobian_diag(P, u0, reciprocal=True))
    if kind == "negjacobi":  # -1 ./ diag(J): SPD for CG on Bratu's negative definite J
        d = -oc.jacobian_diag(P, u0, reciprocal=True)
        return ah.DiagonalPreconditioner(ah.DeviceArray.from_numpy(d.reshape(P.shape))), ("diag", d)
    if kind == "ilu0":
        return ah.ilu0(J), ("ilu0", oc.ilu0_factor(P, u0))
    return ah.GmresPreconditioner(J, kind[1]), ("gmres", kind[1])


@pytest.mark.parametrize("algo,side,kind,nx,ny,kw", [
    ("gmres", "N", "jacobi", 512, 384, dict(restart=True, itmax=60, memory=20)),    # x += N (V y); ||x|| by k_sumsq
    ("fgmres", "N", "jacobi", 512, 384, dict(restart=True, itmax=60, memory=20)),   # Z_k kept, fused x update
    ("gmres", "M", "jacobi", 512, 384, dict(restart=True, itmax=60, memory=20)),    # <V_1, M J V_k> by k_dot
    ("gmres", "N", "ilu0", 256, 192, dict(restart=True, itmax=40, memory=20, ldiv=True)),
    ("fgmres", "N", ("gmres", 5), 256, 192, dict(restart=False, itmax=30, memory=30)),  # inner device GMRES
    ("cg", "M", "negjacobi", 256, 192, dict(itmax=150)),                             # <r, M r> by k_dot
])
def test_preconditioned_solve_bitwise_in_device_order(ctx, algo, side, kind, nx, ny, kw):
    """Krylov.jl gmres! / fgmres! / cg! with N or M against the oracle in the device's
    order: the preconditioner's own reductions too -- ||N V_k|| for the FD step fused into k_diag_apply's
    scalar chunks (k_sumsq after an ILU(0) solve or an inner GMRES), ||M b|| and the restart's ||M r||,
    <V_1, M J V_k> by k_dot, ||x|| by k_sumsq where gmres! applies N after the update.  Equal counts, the
    residual history and x bit for bit (test_hip_precond.py compares these at 1e-8)."""
    P = oc.bratu2d(nx, ny)
    u0 = oc.sin_ic(P) + 0.05 * np.random.default_rng(4).standard_normal(P.shape)
    u = ah.DeviceArray.from_numpy(u0)
    res = u.zero()
    ah.bratu2d_(res, u, (P.hx, P.hy, P.lam))
    J = ah.JacobianOperator(ah.bratu2d_, res, u, (P.hx, P.hy, P.lam), jv="fd")
    dev_p, oc_p = _prec(kind, J, P, u0)
    kw = dict(kw, atol=0.0, rtol=0.0)
    memory = kw.pop("memory", 20)
    ws = ah.krylov_workspace(algo, ah.KrylovConstructor(res, memory=memory))
    ah.krylov_solve_(ws, J, res, history=True, **{side: dev_p}, **kw)
    x, st = ws.x.to_numpy(), ws.stats
    path = ctx.path_info()
    ws.free()
    okw = {k: v for k, v in kw.items() if k != "ldiv"}
    b = res.to_numpy()
    np.testing.assert_array_equal(b, oc.residual(P, u0))
    oc.set_devred(True, cus=path["resident_blocks"] or 256)
    try:
        xo, so, ho = oc.krylov_solve(P, u0, b, algo=algo, jv="fd", F0=b, memory=memory, **{side: oc_p}, **okw)
    finally:
        oc.set_devred(False)
    assert st.niter == so["niter"] and st.n_matvec == so["n_matvec"]
    np.testing.assert_array_equal(np.array(st.residuals), ho)
    np.testing.assert_array_equal(x, xo)


@pytest.mark.parametrize("case", ["gmres_jacobi", "fgmres_inner5", "gmres_left_jacobi", "gmres_ilu"])
def test_newton_preconditioned_bitwise_in_device_order(ctx, case):
    """newton_krylov! with an N / M factory per Newton step (src/Ariadne.jl:318-333) on 2D Bratu, FD Jv,
    against the oracle in the device's order: equal outer / inner / matvec counts, the ||F|| history and the
    root bit for bit (test_hip_precond.py: counts, root to 1e-9)."""
    algo, N, M, tol, kw = {
        "gmres_jacobi": ("gmres", "jacobi", None, 1e-8, dict(memory=20, krylov_kwargs=dict(restart=True))),
        "fgmres_inner5": ("fgmres", ("gmres", 5), None, 1e-8, dict(memory=30)),
        # left: the inner test measures ||M r|| (~h^2 ||r||), so EW stops the inner solves early and Newton
        # stalls near 1e-5 relative (the oracle alike) -- a looser tolerance
        "gmres_left_jacobi": ("gmres", None, "jacobi", 1e-4, dict(memory=20, krylov_kwargs=dict(restart=True))),
        "gmres_ilu": ("gmres", "ilu", None, 1e-8, dict(memory=30, krylov_kwargs=dict(restart=True, ldiv=True))),
    }[case]
    P = oc.bratu2d(128, 96)
    u0 = oc.sin_ic(P)
    fac = {None: None, "jacobi": ah.jacobi, "ilu": ah.ilu0}
    dN = fac[N] if not isinstance(N, tuple) else ah.gmres_preconditioner(N[1])
    hist = []
    u, r = ah.newton_krylov_(ah.bratu2d_, ah.DeviceArray.from_numpy(u0), (P.hx, P.hy, P.lam), algo=algo, jv="fd",
                             N=dN, M=fac[M], tol_rel=tol, callback=lambda u_, res_, n: hist.append(n), **kw)
    path = ctx.path_info()
    okw = dict(memory=kw["memory"], **{k: v for k, v in kw.get("krylov_kwargs", {}).items() if k != "ldiv"})
    oc.set_devred(True, cus=path["resident_blocks"] or 256)
    try:
        uo, so = oc.newton_krylov(P, u0, algo=algo, jv="fd", N=N, M=M, tol_rel=tol, **okw)
    finally:
        oc.set_devred(False)
    assert r.solved and so["solved"]
    assert (r.stats.outer_iterations, r.stats.inner_iterations) == (so["outer_iterations"], so["inner_iterations"])
    assert r.n_matvec == so["n_matvec"]
    np.testing.assert_array_equal(np.array(hist), so["n_res_history"])
    np.testing.assert_array_equal(u.to_numpy(), uo)


@pytest.mark.parametrize("N,algo", [("jacobi", "gmres"), (("gmres", 5), "fgmres")])
def test_newton_preconditioned_config1_bitwise_in_device_order(ctx, N, algo):
    """examples/bratu.jl's preconditioned solves at BASELINE config 1 (1D Bratu N = 1000, exact JVP): the
    inner counts test_hip_precond.py can only hold to 5 % (chaotic in the last bits on cond(J) ~ 1.75e8)
    are equal here, and the root is bit for bit the oracle's."""
    P = oc.bratu1d(1000)
    u0 = oc.sin_ic(P)
    factory = ah.jacobi if N == "jacobi" else ah.gmres_preconditioner(N[1])
    u, r = ah.newton_krylov_(ah.bratu_, ah.DeviceArray.from_numpy(u0), (P.hx, P.lam), N=factory, algo=algo)
    oc.set_devred(True)
    try:
        ref, so = oc.newton_krylov(P, u0, algo=algo, N=N)
    finally:
        oc.set_devred(False)
    assert r.solved and so["solved"]
    assert (r.stats.outer_iterations, r.stats.inner_iterations) == (so["outer_iterations"], so["inner_iterations"])
    assert r.n_matvec == so["n_matvec"]
    np.testing.assert_array_equal(u.to_numpy(), ref)


# ----------------------------------------------------------------------------- implicit.jl schemes, 2D and 3D
_G = {"euler": ah.G_Euler_, "midpoint": ah.G_Midpoint_, "trapezoid": ah.G_Trapezoid_}
_BC = {oc.BC_ZERO: ah.bc_zero_, oc.BC_PERIODIC: ah.bc_periodic_}


@pytest.mark.parametrize("scheme,alpha,bc,shape", [
    ("euler", 0.5, oc.BC_ZERO, (256, 192)),
    ("trapezoid", 0.5, oc.BC_PERIODIC, (256, 256)),     # k_st2d's periodic instance (square: heat_2D.jl:23-24)
    ("midpoint", 0.3, oc.BC_ZERO, (130, 67)),           # odd width: one-column (VEC 1) tiles
    ("euler", 0.5, oc.BC_ZERO, (64, 48, 40)),           # k_st3l's tiles, z-chunks
    ("midpoint", 0.5, oc.BC_PERIODIC, (48, 48, 48)),
    ("trapezoid", 0.5, oc.BC_ZERO, (66, 33, 20)),
])
def test_scheme_newton_bitwise_in_device_order(ctx, scheme, alpha, bc, shape):
    """One implicit step of each implicit.jl scheme (G_Euler! / G_Midpoint!(α) / G_Trapezoid! over diffusion!,
    bc_zero! / bc_periodic!) as the config-3 / config-5 benches run it -- newton_krylov!, tol_abs = 6e-6, FD
    Jv, unrestarted GMRES(20) with reorthogonalisation -- against the oracle in the device's order: equal
    counts, the ||F|| history and the step bit for bit, 2D and 3D (test_hip_schemes.py: to 1e-10)."""
    rng = np.random.default_rng(11)
    un = rng.standard_normal(shape[::-1])
    mk = oc.heat2d_euler if len(shape) == 2 else oc.heat3d_euler
    P = mk(*shape, un=un, scheme=scheme, bc=bc, alpha=alpha)
    G = _G[scheme](alpha=alpha) if scheme == "midpoint" else _G[scheme]
    F = G.bind(ah.diffusion_ if P.dim == 2 else ah.diffusion3d_)
    fp = (P.a, P.hx, P.hy, _BC[bc]) if P.dim == 2 else (P.a, P.hx, P.hy, P.hz, _BC[bc])
    p = (ah.DeviceArray.from_numpy(un), P.dt, None, fp, 0.0)
    u0 = un + 0.01 * rng.standard_normal(un.shape)
    hist = []
    kw = dict(tol_abs=6e-6, jv="fd", krylov_kwargs=dict(reorthogonalization=True))
    u, r = ah.newton_krylov_(F, ah.DeviceArray.from_numpy(u0), p, callback=lambda u_, res_, n: hist.append(n), **kw)
    path = ctx.path_info()
    oc.set_devred(True, cus=path["resident_blocks"] or 256)
    try:
        uo, so = oc.newton_krylov(P, u0, tol_abs=6e-6, jv="fd", reorthogonalization=True)
    finally:
        oc.set_devred(False)
    assert r.solved and so["solved"]
    assert (r.stats.outer_iterations, r.stats.inner_iterations) == (so["outer_iterations"], so["inner_iterations"])
    np.testing.assert_array_equal(np.array(hist), so["n_res_history"])
    np.testing.assert_array_equal(u.to_numpy(), uo)
