"""GPU parity tests: the HIP path (through libnkhip.so's C ABI) against the CPU oracle and the goldens.

Tolerances (stated per test):
  * heat residual / JVP: no transcendental -> bit-identical to the oracle (both -ffp-contract=off,
    same association order).
  * Bratu residual / JVP / FD operator: bit-identical too -- the device and the oracle evaluate
    lambda*exp(u) with the same correctly rounded exp (csrc/nk_exp.h, pinned by tests/test_exp.py).
  * BLAS-1 elementwise ops: bit-identical (same fma convention); dot/norm: 1e-13 relative
    (different, but fixed, summation order).
  * Krylov / Newton: equal iteration counts; residual histories 1e-8 relative over the first cycle;
    converged solutions to the stated solver tolerance.
"""
import json
import os

import numpy as np
import pytest

import _nkpath  # noqa: F401
import ariadne_hip as ah
from oracle import oracle as oc

pytestmark = pytest.mark.gpu

ULP = np.finfo(np.float64).eps


@pytest.fixture(scope="module")
def ctx():
    c = ah.Context(0)
    ah.set_default_context(c)
    yield c
    c.sync()


def dev(a, grid=None):
    return ah.DeviceArray.from_numpy(a, grid)


def params(P):
    if P.kind == oc.BRATU1D:
        return ah.bratu_, (P.hx, P.lam)
    if P.kind == oc.BRATU2D:
        return ah.bratu2d_, (P.hx, P.hy, P.lam)
    un = dev(P.un)
    if P.kind == oc.HEAT2D_EULER:
        return ah.heat2d_euler_, (un, P.dt, None, (P.a, P.hx, P.hy, ah.bc_zero_), 0.0)
    return ah.heat3d_euler_, (un, P.dt, None, (P.a, P.hx, P.hy, P.hz, ah.bc_zero_), 0.0)


def problems():
    rng = np.random.default_rng(11)
    out = []
    for P in (oc.bratu1d(1000), oc.bratu1d(7), oc.bratu2d(64), oc.bratu2d(63, 37), oc.bratu2d(1000, 5),
              oc.bratu2d(1, 1), oc.bratu2d(3, 1), oc.bratu2d(1, 6), oc.bratu2d(130, 9)):
        out.append((P, oc.sin_ic(P) + 0.05 * rng.standard_normal(P.shape)))
    for shape in ((40, 40), (130, 67), (33, 5), (1, 1)):
        un = rng.standard_normal(shape[::-1])
        P = oc.heat2d_euler(*shape, un=un)
        out.append((P, un + 0.01 * rng.standard_normal(un.shape)))
    for shape in ((12, 12, 12), (33, 17, 9), (8, 5, 20), (2, 3, 1)):
        un = rng.standard_normal(shape[::-1])
        P = oc.heat3d_euler(*shape, un=un)
        out.append((P, un + 0.01 * rng.standard_normal(un.shape)))
    return out


PROBLEMS = problems()
IDS = [f"k{P.kind}-{P.nx}x{P.ny}x{P.nz}" for P, _ in PROBLEMS]


def compare(P, got, ref, u):
    assert np.array_equal(got, ref), f"max diff {np.max(np.abs(got - ref))}"


@pytest.mark.parametrize("P,u", PROBLEMS, ids=IDS)
def test_residual_parity(ctx, P, u):
    F, p = params(P)
    ud = dev(u)
    res = ud.zero()
    F(res, ud, p)
    compare(P, res.to_numpy(), oc.residual(P, u), u)
    nrm = F.residual_norm(res, ud, p)
    assert abs(nrm - oc.norm(oc.residual(P, u))) <= 1e-13 * nrm + 1e-300


@pytest.mark.parametrize("P,u", PROBLEMS, ids=IDS)
def test_jv_exact_parity(ctx, P, u):
    F, p = params(P)
    v = np.random.default_rng(3).standard_normal(u.shape)
    ud, vd = dev(u), dev(v)
    res, out = ud.zero(), ud.zero()
    ah.mul_(out, ah.JacobianOperator(F, res, ud, p, jv="exact"), vd)
    np.testing.assert_array_equal(out.to_numpy(), oc.jv_exact(P, u, v))


@pytest.mark.parametrize("P,u", PROBLEMS, ids=IDS)
def test_jv_fd_parity(ctx, P, u):
    F, p = params(P)
    v = np.random.default_rng(4).standard_normal(u.shape)
    ud, vd = dev(u), dev(v)
    res, out = ud.zero(), ud.zero()
    F(res, ud, p)
    F0 = res.to_numpy()  # same F0 on both sides: only F(u + eps v) is recomputed
    eps = oc.fd_eps(oc.norm(u), oc.norm(v))
    ah.mul_(out, ah.JacobianOperator(F, res, ud, p, jv="fd"), vd, eps=eps)
    np.testing.assert_array_equal(out.to_numpy(), oc.jv_fd(P, u, v, F0, eps))
    # and the FD operator approximates the exact JVP
    exact = oc.jv_exact(P, u, v)
    assert np.max(np.abs(out.to_numpy() - exact)) <= 1e-5 * np.max(np.abs(exact))


# (1 << 24) + 3 and (1 << 25) + 1: the wide streaming grid (kRedCap - 2 blocks) with blocks past the
# last chunk and an odd tail element
@pytest.mark.parametrize("n", [1, 2, 7, 1000, 4097, 1 << 20, (1 << 24) + 3, (1 << 25) + 1])
def test_blas1_parity(ctx, n):
    rng = np.random.default_rng(n)
    x, y = rng.standard_normal(n), rng.standard_normal(n)
    g = ah.Grid.full(n)
    xd, yd = dev(x, g), dev(y, g)
    assert abs(ah.kdot(n, xd, yd) - np.dot(x, y)) <= 1e-13 * np.sqrt(n) * np.linalg.norm(x) * np.linalg.norm(y)
    assert abs(ah.knorm(n, xd) - np.linalg.norm(x)) <= 1e-13 * np.linalg.norm(x)
    s, t = 0.37, -1.25
    assert np.array_equal(ah.kaxpy_(n, s, xd, yd.copy()).to_numpy(), oc.axpy(s, x, y))
    assert np.array_equal(ah.kaxpby_(n, s, xd, t, yd.copy()).to_numpy(), oc.axpby(s, x, t, y))
    assert np.array_equal(ah.kscal_(n, s, xd.copy()).to_numpy(), s * x)
    assert np.array_equal(ah.kdivcopy_(n, yd.copy(), xd, 3.0).to_numpy(), x / 3.0)
    assert np.array_equal(ah.kcopy_(n, yd.copy(), xd).to_numpy(), x)
    assert np.array_equal(ah.kfill_(xd.copy(), 2.5).to_numpy(), np.full(n, 2.5))
    a, b = ah.kref_(n, xd.copy(), yd.copy(), 0.6, 0.8)
    assert np.array_equal(a.to_numpy(), 0.6 * x + 0.8 * y)
    assert np.array_equal(b.to_numpy(), 0.8 * x - 0.6 * y)


def test_dot_deterministic(ctx):
    n = 3_000_001
    rng = np.random.default_rng(5)
    x, y = rng.standard_normal(n), rng.standard_normal(n)
    g = ah.Grid.full(n)
    xd, yd = dev(x, g), dev(y, g)
    vals = {ah.kdot(n, xd, yd) for _ in range(5)}
    assert len(vals) == 1


# ----------------------------------------------------------------------------- Krylov solves
def devred_solve(P, u, b, cus=256, **kw):
    """The oracle's solve in the device's reduction order (oracle.set_devred, test_hip_devred.py)."""
    oc.set_devred(True, cus=cus)
    try:
        return oc.krylov_solve(P, u, b, **kw)
    finally:
        oc.set_devred(False)


def device_solve(P, u, b, **kw):
    F, p = params(P)
    ud, bd = dev(u), dev(b)
    res = ud.zero()
    F(res, ud, p)
    algo = kw.pop("algo", "gmres")
    jv = kw.pop("jv", "exact")
    memory = kw.pop("memory", 20)
    ws = ah.krylov_workspace(algo, ah.KrylovConstructor(res, memory=memory))
    J = ah.JacobianOperator(F, res, ud, p, jv=jv)
    ah.krylov_solve_(ws, J, bd, history=True, **kw)
    return ws.x.to_numpy(), ws.stats, res.to_numpy()


@pytest.mark.parametrize("restart,memory,reorth,jv", [(False, 20, False, "exact"), (True, 10, False, "exact"),
                                                      (True, 8, True, "exact"), (True, 10, False, "fd")])
def test_gmres_matches_oracle(ctx, restart, memory, reorth, jv):
    P = oc.bratu2d(24)
    u = oc.sin_ic(P)
    b = oc.residual(P, u)
    kw = dict(restart=restart, reorthogonalization=reorth, atol=1e-12, rtol=1e-9, itmax=150)
    x, st, F0 = device_solve(P, u, b, memory=memory, jv=jv, **kw)
    xo, sto, ho = oc.krylov_solve(P, u, b, jv=jv, F0=F0, memory=memory, **kw)
    assert st.niter == sto["niter"] and st.solved == sto["solved"]
    assert st.n_matvec == sto["n_matvec"]
    h = np.array(st.residuals)
    if jv == "exact":
        assert np.allclose(h[: memory + 1], ho[: memory + 1], rtol=1e-8, atol=0)
        m = ho > 1e-6 * ho[0]
        assert np.allclose(h[m], ho[m], rtol=1e-5)
        assert np.max(np.abs(x - xo)) <= 1e-7 * np.max(np.abs(xo))
    else:
        # The FD operator is bit-identical to the oracle's (shared exp), so only the dot / norm summation
        # order separates the two solves, as for heat (test_heat_fd_gmres_matches_oracle).  Measured
        # (tools/bratu_parity_probe.py): first cycle 1.2e-14, the 15-restart history 3.0e-9, x 7.2e-12.
        # (Before the shared exp, ocml's vs glibc's exp moved this history by ~4e-3 and x by ~1e-7.)
        assert np.allclose(h[: memory + 1], ho[: memory + 1], rtol=1e-12, atol=0)
        k = ho > 1e-6 * ho[0]
        assert np.allclose(h[k], ho[k], rtol=1e-8, atol=0)
        assert np.max(np.abs(x - xo)) <= 1e-10 * np.max(np.abs(xo))
    # in the device's reduction order the same restatement is bit for bit
    xr, sr, hr = devred_solve(P, u, b, jv=jv, F0=F0, memory=memory, **kw)
    assert sr["niter"] == st.niter
    np.testing.assert_array_equal(h, hr)
    np.testing.assert_array_equal(x, xr)


@pytest.mark.parametrize("restart,memory", [(True, 10), (False, 20)])
def test_heat_fd_gmres_matches_oracle(ctx, restart, memory):
    """FD-GMRES on a heat residual (G_Euler! of heat_2D.jl: no exp, so F agrees bit for bit): only the
    reductions' summation order separates the GPU from the oracle -- histories to 1e-9, x to 1e-11."""
    n = 24
    u0 = oc.sin_ic(oc.bratu2d(n)) + 0.1 * np.random.default_rng(1).standard_normal((n, n))
    un = u0.copy()
    P = oc.heat2d_euler(n, un=un)
    u = u0 + 0.01
    b = oc.residual(P, u)
    kw = dict(restart=restart, atol=1e-12, rtol=1e-9, itmax=150)
    x, st, F0 = device_solve(P, u, b, memory=memory, jv="fd", **kw)
    np.testing.assert_array_equal(F0, b)  # the heat residual is bit-identical
    xo, so, ho = oc.krylov_solve(P, u, b, jv="fd", F0=F0, memory=memory, **kw)
    assert st.niter == so["niter"] and st.n_matvec == so["n_matvec"]
    h = np.array(st.residuals)
    k = ho > 1e-6 * ho[0]
    assert np.allclose(h[k], ho[k], rtol=1e-9, atol=0)
    assert np.max(np.abs(x - xo)) <= 1e-11 * np.max(np.abs(xo))
    xr, _, hr = devred_solve(P, u, b, jv="fd", F0=F0, memory=memory, **kw)
    np.testing.assert_array_equal(h, hr)
    np.testing.assert_array_equal(x, xr)


def test_cg_matches_oracle(ctx):
    P = oc.bratu1d(300)
    u = oc.sin_ic(P)
    b = oc.residual(P, u)
    x, st, _ = device_solve(P, u, b, algo="cg", atol=1e-12, rtol=1e-10)
    xo, sto, ho = oc.krylov_solve(P, u, b, algo="cg", atol=1e-12, rtol=1e-10)
    assert st.niter == sto["niter"]
    m = ho > 1e-6 * ho[0]
    assert np.allclose(np.array(st.residuals)[m], ho[m], rtol=1e-6)
    assert np.max(np.abs(x - xo)) <= 1e-6 * np.max(np.abs(xo))
    xr, _, hr = devred_solve(P, u, b, algo="cg", atol=1e-12, rtol=1e-10)
    np.testing.assert_array_equal(np.array(st.residuals), hr)
    np.testing.assert_array_equal(x, xr)


def test_gmres_deterministic(ctx):
    P = oc.bratu2d(48)
    u = oc.sin_ic(P)
    b = oc.residual(P, u)
    xs = [device_solve(P, u, b, restart=True, memory=10, itmax=40, atol=0.0, rtol=0.0)[0] for _ in range(2)]
    assert np.array_equal(xs[0], xs[1])


# ----------------------------------------------------------------------------- Newton (Ariadne)
def test_newton_bratu1d_cg_config1(ctx, golden_dir):
    """BASELINE config 1: examples/bratu.jl:59-63 (N = 1000, algo = :cg) -- solved, same stats as the oracle."""
    g = np.load(os.path.join(golden_dir, "bratu1d_n1000.npz"))
    P = oc.bratu1d(1000)
    u = dev(g["u0"])
    u, r = ah.newton_krylov_(ah.bratu_, u, (P.hx, P.lam), u.similar(), algo="cg")
    uo, so = oc.newton_krylov(P, g["u0"], algo="cg")
    assert r.solved and so["solved"]
    assert abs(r.stats.outer_iterations - so["outer_iterations"]) <= 1
    # thousands of CG iterations on cond(J) ~ 1.75e8: counts are chaotic in the last bits (a 1-ulp
    # change of u0 moves the oracle's own count by ~9%), so only the outcome is compared
    assert abs(r.stats.inner_iterations - so["inner_iterations"]) <= 0.15 * so["inner_iterations"]
    assert np.max(np.abs(u.to_numpy() - g["true_sol"])) < 3e-4


def test_newton_bratu2d_gmres30_golden(ctx, golden_dir):
    g = np.load(os.path.join(golden_dir, "bratu2d_64.npz"))
    P = oc.bratu2d(64)
    u = dev(g["u0"])
    kw = dict(restart=True)
    u, r = ah.newton_krylov_(ah.bratu2d_, u, (P.hx, P.hy, P.lam), memory=30, tol_rel=1e-10, krylov_kwargs=kw)
    uo, so = oc.newton_krylov(P, g["u0"], memory=30, restart=True, tol_rel=1e-10)
    assert r.solved
    assert r.stats.outer_iterations == so["outer_iterations"]
    assert r.stats.inner_iterations == so["inner_iterations"]
    assert np.max(np.abs(u.to_numpy() - g["ustar"])) <= 1e-8 * np.max(np.abs(g["ustar"]))
    oc.set_devred(True)  # the oracle in the device's reduction order: the root bit for bit
    try:
        ud, _ = oc.newton_krylov(P, g["u0"], memory=30, restart=True, tol_rel=1e-10)
    finally:
        oc.set_devred(False)
    np.testing.assert_array_equal(u.to_numpy(), ud)
    # same ||F(u)|| as the CPU path on the same final iterate: F itself is bit-identical, only the
    # norm's summation order differs
    uu = u.to_numpy()
    Fcpu = oc.residual(P, uu)
    assert abs(oc.norm(Fcpu) - r.stats.n_res) <= 1e-13 * oc.norm(Fcpu)
    # away from the floor (after 2 Newton steps) the north-star 1e-10 relative statement holds
    u2, r2 = ah.newton_krylov_(ah.bratu2d_, dev(g["u0"]), (P.hx, P.hy, P.lam), memory=30, max_niter=1,
                               tol_rel=0.0, tol_abs=0.0, krylov_kwargs=kw)
    F2 = oc.norm(oc.residual(P, u2.to_numpy()))
    assert r2.stats.outer_iterations == 2
    assert abs(F2 - r2.stats.n_res) <= 1e-10 * F2


def test_newton_bratu2d_256_scipy_root(ctx):
    """SURVEY §8c's independent root oracle at 256^2: a scipy sparse-direct Newton iteration
    (tests/golden/make_golden.py's numpy residual and assembled Jacobian, computed here rather than
    stored) against the device Newton-Krylov root -- ILU(0)-preconditioned GMRES(30), restarted, as
    examples/bratu.jl:119-137 preconditions -- to 1e-8 of max |u| (||F|| <= 1e-11 ||F(u0)||, cond(J)
    ~ 1e4), and ||F|| of the device root (on the oracle's residual) at the solve's tolerance."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_golden as mg
    import scipy.sparse as sp

    n = 256
    P = oc.bratu2d(n)
    u0 = oc.sin_ic(P)
    h = P.hx
    F = lambda u: (mg.d2(u, 1, h) + mg.d2(u, 0, h)) + mg.LAM * np.exp(u)  # noqa: E731
    L = sp.kronsum(mg.lap1d(n, h), mg.lap1d(n, h))
    ustar, hist = mg.newton_sparse(F, lambda u: L + sp.diags(mg.LAM * np.exp(u.ravel())), u0.copy(), tol=1e-9)
    assert hist[-1] < 1e-9
    u, r = ah.newton_krylov_(ah.bratu2d_, dev(u0), (P.hx, P.hy, P.lam), N=ah.ilu0, memory=30, tol_rel=1e-11,
                             krylov_kwargs={"restart": True, "ldiv": True, "atol": 1e-15})
    # (Krylov.jl's default atol = sqrt(eps) would stop every inner solve once ||F|| < 1.5e-8)
    assert r.solved, (r.stats, r.n_res_history if hasattr(r, "n_res_history") else None)
    got = u.to_numpy()
    assert np.max(np.abs(got - ustar)) <= 1e-8 * np.max(np.abs(ustar))
    assert oc.norm(oc.residual(P, got)) <= 2e-11 * oc.norm(oc.residual(P, u0))


def test_newton_fd_vs_exact(ctx):
    P = oc.bratu2d(32)
    u0 = oc.sin_ic(P)
    p = (P.hx, P.hy, P.lam)
    kw = dict(restart=True)
    ue, re_ = ah.newton_krylov_(ah.bratu2d_, dev(u0), p, memory=30, tol_rel=1e-9, krylov_kwargs=kw, jv="exact")
    uf, rf = ah.newton_krylov_(ah.bratu2d_, dev(u0), p, memory=30, tol_rel=1e-9, krylov_kwargs=kw, jv="fd")
    uo, so = oc.newton_krylov(P, u0, memory=30, restart=True, tol_rel=1e-9, jv="fd")
    assert re_.solved and rf.solved
    assert rf.stats.outer_iterations == so["outer_iterations"]
    assert np.max(np.abs(uf.to_numpy() - ue.to_numpy())) <= 1e-8 * np.max(np.abs(ue.to_numpy()))
    oc.set_devred(True)
    try:
        for jv, ud in (("fd", uf), ("exact", ue)):  # each operator's solve bit for bit in the device's order
            uo, _ = oc.newton_krylov(P, u0, memory=30, restart=True, tol_rel=1e-9, jv=jv)
            np.testing.assert_array_equal(ud.to_numpy(), uo)
    finally:
        oc.set_devred(False)


def test_newton_forcing_variants_and_outofplace(ctx):
    P = oc.bratu2d(32)
    u0 = oc.sin_ic(P)
    p = (P.hx, P.hy, P.lam)
    for forcing, name in ((ah.Fixed(0.1), "fixed"), (None, "none"), (ah.EisenstatWalker(), "ew")):
        u, r = ah.newton_krylov_(ah.bratu2d_, dev(u0), p, memory=30, forcing=forcing, krylov_kwargs=dict(restart=True))
        uo, so = oc.newton_krylov(P, u0, memory=30, restart=True, forcing=name)
        assert r.solved and so["solved"]
        assert r.stats.outer_iterations == so["outer_iterations"]
        oc.set_devred(True)
        try:
            ud, sd = oc.newton_krylov(P, u0, memory=30, restart=True, forcing=name)
        finally:
            oc.set_devred(False)
        assert r.stats.inner_iterations == sd["inner_iterations"]
        np.testing.assert_array_equal(u.to_numpy(), ud)
    ud = dev(u0)
    u2, r2 = ah.newton_krylov(ah.bratu2d_, ud, p, memory=30, krylov_kwargs=dict(restart=True))
    assert r2.solved and np.array_equal(ud.to_numpy(), u0)  # out-of-place leaves u0 alone


def test_heat2d_reference_ic_step(ctx, golden_dir):
    """heat_2D.jl IC = Laplacian eigenvector: one implicit Euler step is an exact decay, 1 Krylov iteration."""
    g = np.load(os.path.join(golden_dir, "heat2d_40.npz"))
    un = dev(g["u0"])
    u = un.copy()
    p = (un, float(g["dt"]), None, (float(g["a"]), float(g["dx"]), float(g["dx"]), ah.bc_zero_), 0.0)
    u, r = ah.newton_krylov_(ah.heat2d_euler_, u, p, tol_abs=6e-6)
    assert r.solved and r.stats.inner_iterations == 1
    assert np.max(np.abs(u.to_numpy() - g["u1"])) < 1e-10


def test_heat2d_solve_timestepping(ctx):
    """implicit.jl `solve` with G_Euler! on a noisy IC: per-step Newton/Krylov counts equal the oracle's."""
    N = 64
    rng = np.random.default_rng(0)
    P = oc.heat2d_euler(N)
    u0 = oc.sin_ic(P) + 0.1 * rng.uniform(-1, 1, (N, N))
    ts = [i * P.dt for i in range(4)]
    un = dev(u0)
    results = []
    ah.solve(ah.G_Euler_, ah.diffusion_, un, (P.a, P.hx, P.hy, ah.bc_zero_), P.dt, ts, stats_out=results)
    cur = u0.copy()
    for r in results:
        Q = oc.heat2d_euler(N, un=cur)
        cur, so = oc.newton_krylov(Q, cur, tol_abs=6e-6)
        assert r.solved and so["solved"]
        assert (r.stats.outer_iterations, r.stats.inner_iterations) == (so["outer_iterations"], so["inner_iterations"])
    assert np.max(np.abs(un.to_numpy() - cur)) <= 1e-10
    cur = u0.copy()  # the time loop in the device's reduction order: bit for bit
    oc.set_devred(True)
    try:
        for _ in results:
            cur, _ = oc.newton_krylov(oc.heat2d_euler(N, un=cur), cur, tol_abs=6e-6)
    finally:
        oc.set_devred(False)
    np.testing.assert_array_equal(un.to_numpy(), cur)


def test_heat3d_newton(ctx, golden_dir):
    g = np.load(os.path.join(golden_dir, "heat3d_12.npz"))
    P = oc.heat3d_euler(12, un=g["un"])
    F, p = params(P)
    u, r = ah.newton_krylov_(F, dev(g["u"]), p, tol_abs=6e-6)
    uo, so = oc.newton_krylov(P, g["u"], tol_abs=6e-6)
    assert r.solved and (r.stats.outer_iterations, r.stats.inner_iterations) == (so["outer_iterations"], so["inner_iterations"])
    assert np.max(np.abs(u.to_numpy() - uo)) <= 1e-12
    oc.set_devred(True)
    try:
        ud, _ = oc.newton_krylov(P, g["u"], tol_abs=6e-6)
    finally:
        oc.set_devred(False)
    np.testing.assert_array_equal(u.to_numpy(), ud)


# ----------------------------------------------------------------------------- BASELINE size (4096^2)
def test_bratu2d_4096_full_size(ctx):
    """Config 2 size: kernels vs the oracle, exact-JVP linearity, and the first GMRES(30) steps."""
    n = 4096
    P = oc.bratu2d(n)
    u = oc.sin_ic(P)
    v = np.random.default_rng(9).standard_normal(u.shape)
    F, p = params(P)
    ud, vd = dev(u), dev(v)
    res, out, out2 = ud.zero(), ud.zero(), ud.zero()
    F(res, ud, p)
    F0 = oc.residual(P, u)
    np.testing.assert_array_equal(res.to_numpy(), F0)
    J = ah.JacobianOperator(F, res, ud, p, jv="exact")
    ah.mul_(out, J, vd)
    np.testing.assert_array_equal(out.to_numpy(), oc.jv_exact(P, u, v))
    eps = oc.fd_eps(oc.norm(u), oc.norm(v))
    ah.mul_(out2, ah.JacobianOperator(F, res, ud, p, jv="fd"), vd, eps=eps)
    np.testing.assert_array_equal(out2.to_numpy(), oc.jv_fd(P, u, v, F0, eps))
    # linearity is exact in binary floating point for a power-of-two scale
    ah.kscal_(len(vd), 2.0, vd)
    ah.mul_(out2, J, vd)
    assert np.array_equal(out2.to_numpy(), 2.0 * out.to_numpy())
    # 12 Arnoldi steps of the FD GMRES(30) against the oracle
    kw = dict(restart=True, atol=0.0, rtol=0.0, itmax=12)
    x, st, F0d = device_solve(P, u, F0, memory=30, jv="fd", **kw)
    xo, sto, ho = oc.krylov_solve(P, u, F0, jv="fd", F0=F0d, memory=30, **kw)
    assert st.niter == sto["niter"] == 12
    assert np.allclose(np.array(st.residuals), ho, rtol=1e-8)
    assert np.max(np.abs(x - xo)) <= 1e-8 * np.max(np.abs(xo))
    xr, _, hr = devred_solve(P, u, F0, cus=ctx.path_info()["resident_blocks"] or 256, jv="fd", F0=F0d, memory=30, **kw)
    np.testing.assert_array_equal(np.array(st.residuals), hr)  # the resident sweep's tree at 4096^2: bitwise
    np.testing.assert_array_equal(x, xr)


def test_errors_are_reported(ctx):
    u = dev(np.zeros((4, 4)))
    bad = ah.ariadne.JacobianOperator(ah.bratu2d_, u.zero(), u, (0.1, 0.1, 1.0))
    with pytest.raises(ValueError):
        ah.bratu_(u.zero(), u, (0.1, 1.0))  # 1D residual on a 2D grid
    ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(dev(np.zeros((5, 5)))))
    with pytest.raises(ah.NKError):
        ah.krylov_solve_(ws, bad, u)  # size mismatch with the workspace
