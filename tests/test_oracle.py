"""Pin the CPU oracle before trusting it (CPU only).

1. the reference's own known answers (test/runtests.jl) through the dual-number restatement;
2. the C oracle's residuals / JVPs against the independent numpy goldens (tests/golden/);
3. the two restatements of the Krylov.jl + Ariadne loop (C and Python) against each other;
4. whole Newton solves against sparse-direct roots, the analytic 1D Bratu solution
   (examples/bratu.jl:33-37) and the exact implicit-Euler decay of the heat eigenvector.
"""
import json
import math
import os

import numpy as np
import pytest

from oracle import ariadne_ref as ar
from oracle import oracle as oc


def _rel(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b))) / max(1e-300, np.max(np.abs(b))))


# ----------------------------------------------------------------------------- runtests.jl known answers
def kelley_F_(res, x, _):
    res[0] = x[0] ** 2 + x[1] ** 2 - 2
    res[1] = ar.dexp(x[0] - 1) + x[1] ** 2 - 2


def kelley_F(x, p):
    res = np.zeros(2, dtype=object) if x.dtype == object else np.zeros(2)
    kelley_F_(res, x, p)
    return res


@pytest.fixture(scope="module")
def kelley(golden_dir):
    with open(os.path.join(golden_dir, "kelley2x2.json")) as f:
        return json.load(f)


def test_kelley_jvp_exact(kelley):
    # runtests.jl:36-38: mul!(out, J, [1,0]) == [6.0, 7.38905609893065] (exact equality)
    _, out = ar.jvp(kelley_F_, np.array(kelley["x_jvp"]), np.array([1.0, 0.0]))
    assert list(out) == kelley["jvp_e1"]


def test_kelley_vjp_and_collect(kelley):
    x = np.array(kelley["x_jvp"])
    assert list(ar.vjp(kelley_F_, x, [1.0, 0.0])) == kelley["vjp_e1"]      # runtests.jl:40-42
    J = ar.collect(kelley_F_, x)
    assert np.array_equal(J, np.array(kelley["jacobian"]))                  # runtests.jl:44-46
    assert np.array_equal(ar.collect(kelley_F_, x).T, J.T)                  # runtests.jl:54
    v = np.random.default_rng(0).random(2)
    assert np.allclose(ar.jvp(kelley_F_, x, v)[1], J @ v)                   # runtests.jl:48-52


def test_kelley_newton_solved(kelley):
    for x0 in kelley["starts_inplace"]:                                     # runtests.jl:15-18
        x, st = ar.newton_krylov_(kelley_F_, np.array(x0))
        assert st["solved"]
        assert np.allclose(x, kelley["root"], atol=1e-5)
    for x0 in kelley["starts_outofplace"]:                                  # runtests.jl:20-23
        x, st = ar.newton_krylov(kelley_F, np.array(x0))
        assert st["solved"]


# ----------------------------------------------------------------------------- forcing / givens
def test_eisenstat_walker_matches_c():
    ew = ar.EisenstatWalker()
    rng = np.random.default_rng(5)
    for _ in range(200):
        eta, tol = rng.uniform(0, 1), 10 ** rng.uniform(-12, -2)
        n_prior = 10 ** rng.uniform(-6, 2)
        n = n_prior * rng.uniform(0.01, 1.2)
        assert ew(eta, tol, n, n_prior) == oc.ew_forcing(eta, tol, n, n_prior)


def test_eisenstat_walker_rational_threshold():
    # γη² exactly equal to the double 0.1 is NOT <= 1//10 (the double 0.1 exceeds 1/10):
    ew = ar.EisenstatWalker(eta_max=0.999, gamma=1.0)
    eta = math.sqrt(0.1)
    g_eta2 = 1.0 * eta ** 2
    n_res, n_prior, tol = 1e-3, 1.0, 1e-12
    expect = (min(0.999, max(0.9 * 0 + n_res ** 2 / n_prior ** 2, g_eta2)) if g_eta2 >= 0.1
              else min(0.999, n_res ** 2 / n_prior ** 2))
    assert ew(eta, tol, n_res, n_prior) == max(expect, 0.5 * tol / n_res)


def test_sym_givens():
    for a, b in [(3.0, 4.0), (-2.0, 0.5), (0.0, 0.0), (0.0, -3.0), (1.5, 0.0), (1e-300, 1e300)]:
        c, s, r = oc.sym_givens(a, b)
        assert (c, s, r) == ar.sym_givens(a, b)
        assert abs(c * a + s * b - r) <= 1e-14 * max(1.0, abs(r))
        if a != 0 or b != 0:
            assert abs(s * a - c * b) <= 1e-14 * max(abs(a), abs(b))


# ----------------------------------------------------------------------------- kernels vs numpy goldens
def test_bratu1d_kernels(golden_dir):
    g = np.load(os.path.join(golden_dir, "bratu1d_n1000.npz"))
    P = oc.bratu1d(1000)
    assert P.hx == g["dx"]
    assert np.array_equal(oc.sin_ic(P), np.sin(g["x"] * np.pi)) or _rel(oc.sin_ic(P), g["u0"]) < 1e-15
    u0 = g["u0"]
    assert _rel(oc.residual(P, u0), g["F0"]) < 1e-14
    assert _rel(oc.jv_exact(P, u0, g["v"]), g["Jv"]) < 1e-14
    # FD operator approximates the exact JVP to ~sqrt(eps)
    assert _rel(oc.jv_fd(P, u0, g["v"]), g["Jv"]) < 1e-6


def test_bratu2d_kernels(golden_dir):
    g = np.load(os.path.join(golden_dir, "bratu2d_64.npz"))
    P = oc.bratu2d(64)
    assert _rel(oc.sin_ic(P), g["u0"]) < 1e-15
    assert _rel(oc.residual(P, g["u0"]), g["F0"]) < 1e-14
    assert _rel(oc.jv_exact(P, g["u0"], g["v"]), g["Jv"]) < 1e-14
    assert _rel(oc.jv_fd(P, g["u0"], g["v"]), g["Jv"]) < 1e-6


def test_heat2d_kernels(golden_dir):
    g = np.load(os.path.join(golden_dir, "heat2d_40.npz"))
    P = oc.heat2d_euler(40, un=g["u0"])
    assert P.dt == g["dt"]
    assert _rel(oc.residual(P, g["u0"]), g["G0"]) < 1e-13
    assert _rel(oc.jv_exact(P, g["u0"], g["v"]), g["Jv"]) < 1e-14
    assert _rel(oc.jv_fd(P, g["u0"], g["v"]), g["Jv"]) < 1e-6


def test_heat3d_kernels(golden_dir):
    g = np.load(os.path.join(golden_dir, "heat3d_12.npz"))
    P = oc.heat3d_euler(12, un=g["un"])
    assert abs(P.dt - g["dt"]) <= 1e-15 * g["dt"]
    assert _rel(oc.residual(P, g["u"]), g["G"]) < 1e-13
    assert _rel(oc.jv_exact(P, g["u"], g["v"]), g["Jv"]) < 1e-14


# ----------------------------------------------------------------------------- Krylov: C vs Python restatement
@pytest.mark.parametrize("restart,memory,reorth", [(False, 20, False), (True, 10, False), (True, 8, True)])
def test_gmres_c_matches_python(restart, memory, reorth):
    P = oc.bratu2d(12)
    u = oc.sin_ic(P)
    b = oc.residual(P, u)
    kw = dict(memory=memory, restart=restart, reorthogonalization=reorth, atol=1e-12, rtol=1e-10, itmax=120)
    x_c, st_c, h_c = oc.krylov_solve(P, u, b, **kw)
    A = lambda v: oc.jv_exact(P, u, v.reshape(P.shape)).ravel()
    x_p, st_p, h_p = ar.gmres(A, b.ravel(), **kw)
    assert st_c["niter"] == st_p.niter and st_c["solved"] == st_p.solved
    # first cycle agrees to rounding; restart residuals amplify rounding at the 1e-8 level later on
    assert np.allclose(h_c[: memory + 1], h_p[: memory + 1], rtol=1e-8, atol=0)
    # rounding differences (different dot order) grow once the residual nears the rounding floor
    h_p = np.asarray(h_p)
    m = h_p > 1e-6 * h_p[0]
    assert np.allclose(h_c[m], h_p[m], rtol=1e-5, atol=0)
    assert _rel(x_c.ravel(), x_p) < 1e-8
    nmv = st_p.niter + (0 if not restart else (st_p.niter - 1) // memory)
    assert st_c["n_matvec"] == nmv


def test_cg_c_matches_python():
    P = oc.bratu1d(200)
    u = oc.sin_ic(P)
    b = oc.residual(P, u)
    x_c, st_c, h_c = oc.krylov_solve(P, u, b, algo="cg", atol=1e-12, rtol=1e-10)
    A = lambda v: oc.jv_exact(P, u, v)
    x_p, st_p, h_p = ar.cg(A, b.copy(), atol=1e-12, rtol=1e-10)
    assert st_c["niter"] == st_p.niter
    assert _rel(x_c, x_p) < 1e-6


def test_gmres_solves_linear_system():
    P = oc.bratu2d(16)
    u = oc.sin_ic(P)
    b = oc.residual(P, u)
    x, st, _ = oc.krylov_solve(P, u, b, atol=0.0, rtol=1e-12, itmax=0)
    assert st["solved"]
    assert oc.norm(oc.jv_exact(P, u, x) - b) <= 1e-10 * oc.norm(b)


# ----------------------------------------------------------------------------- whole Newton solves
def test_newton_bratu1d_cg_matches_root(golden_dir):
    """examples/bratu.jl:59-63 (algo = :cg) at BASELINE config 1 (N = 1000)."""
    g = np.load(os.path.join(golden_dir, "bratu1d_n1000.npz"))
    P = oc.bratu1d(1000)
    u, st = oc.newton_krylov(P, g["u0"], algo="cg")
    assert st["solved"]
    assert st["n_res"] <= st["tol"]
    # discretisation error vs the analytic solution (SURVEY.md §6 probe: 2.6e-4)
    assert np.max(np.abs(u - g["true_sol"])) < 3e-4
    # the discrete root (sparse-direct Newton): cond(J) ~ 1.75e8 => fp64 fixes u only to ~1e-6 here
    assert np.max(np.abs(u - g["ustar"])) < 1e-4


def test_newton_bratu1d_forcing_variants():
    # bratu.jl:92-108: Fixed(0.1) and forcing = nothing (N = 1000; smaller grids stagnate near the fold)
    P = oc.bratu1d(1000)
    u0 = oc.sin_ic(P)
    for forcing in ("ew", "fixed", "none"):
        u, st = oc.newton_krylov(P, u0, algo="cg", forcing=forcing)
        assert st["solved"], forcing


def test_newton_bratu2d_gmres30_matches_root(golden_dir):
    g = np.load(os.path.join(golden_dir, "bratu2d_64.npz"))
    P = oc.bratu2d(64)
    u, st = oc.newton_krylov(P, g["u0"], memory=30, restart=True, tol_rel=1e-10)
    assert st["solved"]
    assert _rel(u, g["ustar"]) < 1e-8


def test_newton_bratu2d_fd_matches_exact():
    P = oc.bratu2d(32)
    u0 = oc.sin_ic(P)
    # tol_rel = 1e-9 keeps tol above Krylov's default atol = sqrt(eps) floor
    ue, se = oc.newton_krylov(P, u0, memory=30, restart=True, tol_rel=1e-9, jv="exact")
    uf, sf = oc.newton_krylov(P, u0, memory=30, restart=True, tol_rel=1e-9, jv="fd")
    assert se["solved"] and sf["solved"]
    assert _rel(uf, ue) < 1e-8
    assert se["outer_iterations"] == sf["outer_iterations"]


def test_newton_matches_python_restatement():
    P = oc.bratu2d(10)
    u0 = oc.sin_ic(P)
    u_c, st_c = oc.newton_krylov(P, u0, memory=20, restart=True)

    h = P.hx

    def F_(res, u, p):  # 2D Bratu written elementwise so the dual numbers differentiate it
        U = u.reshape(P.shape)
        R = res.reshape(P.shape)
        for j in range(P.ny):
            for i in range(P.nx):
                e = U[j, i + 1] if i + 1 < P.nx else 0.0
                w = U[j, i - 1] if i > 0 else 0.0
                n = U[j + 1, i] if j + 1 < P.ny else 0.0
                s = U[j - 1, i] if j > 0 else 0.0
                c = U[j, i]
                R[j, i] = ((e - 2.0 * c) + w) / (h * h) + ((n - 2.0 * c) + s) / (h * h) + oc.LAMBDA_BRATU * ar.dexp(c)

    u_p, st_p = ar.newton_krylov_(F_, u0.ravel(), krylov_kwargs=dict(restart=True), memory=20)
    assert st_c["outer_iterations"] == st_p["outer_iterations"]
    assert st_c["inner_iterations"] == st_p["inner_iterations"]
    assert _rel(u_c.ravel(), u_p) < 1e-9


def test_heat2d_reference_ic_one_step(golden_dir):
    """Reference IC is the discrete Laplacian's eigenvector: one implicit Euler step (tol_abs=6e-6,
    implicit.jl:67-70) must reproduce the exact decay with a single Krylov iteration."""
    g = np.load(os.path.join(golden_dir, "heat2d_40.npz"))
    P = oc.heat2d_euler(40, un=g["u0"])
    u, st = oc.newton_krylov(P, g["u0"], tol_abs=6e-6)
    assert st["solved"]
    assert st["inner_iterations"] == 1
    assert np.max(np.abs(u - g["u1"])) < 1e-10
    assert np.max(np.abs(u - g["decay"] * g["u0"])) < 1e-10


# ----------------------------------------------------------------------------- time-stepping schemes (§8f rank 1)
SCHEMES = [("euler", ar.G_Euler_h, {}), ("midpoint", ar.G_Midpoint_h, {}),
           ("midpoint", ar.G_Midpoint_h, {"alpha": 0.3}), ("trapezoid", ar.G_Trapezoid_h, {})]


@pytest.mark.parametrize("bc", [oc.BC_ZERO, oc.BC_PERIODIC])
@pytest.mark.parametrize("scheme,G,kw", SCHEMES, ids=["euler", "midpoint", "midpoint_a0.3", "trapezoid"])
def test_heat_schemes_match_halo_restatement(scheme, G, kw, bc):
    """The C oracle's G! ∘ diffusion! (all three implicit.jl schemes, bc_zero! / bc_periodic!) against
    a literal restatement of implicit.jl:8-37 + heat_2D.jl:15-62 on halo arrays, differentiated by
    dual numbers: residual and exact JVP bit for bit (square grid: the reference's bc! reuse N for
    the second axis, heat_2D.jl:23-24, 35-36)."""
    rng = np.random.default_rng(7)
    N = 12
    un, u, v = (rng.standard_normal((N, N)) for _ in range(3))
    P = oc.heat2d_euler(N, un=un, scheme=scheme, bc=bc, alpha=kw.get("alpha", 0.5))
    bch = ar.bc_periodic_h if bc == oc.BC_PERIODIC else ar.bc_zero_h
    val, tan = ar.heat_halo_jvp(G, un, u, v, P.a, P.hx, P.hy, P.dt, bch, **kw)
    assert np.array_equal(oc.residual(P, u), val)
    assert np.array_equal(oc.jv_exact(P, u, v), tan)
    assert _rel(oc.jv_fd(P, u, v), tan) < 1e-6


def _decay(scheme, dt, mu, alpha=0.5):
    """Exact one-step amplification of an eigenvector of the discrete Laplacian (eigenvalue mu)."""
    if scheme == "euler":
        return 1.0 / (1.0 - dt * mu)
    if scheme == "midpoint":
        return (1.0 + alpha * dt * mu) / (1.0 - (1.0 - alpha) * dt * mu)
    return (1.0 + 0.5 * dt * mu) / (1.0 - 0.5 * dt * mu)


@pytest.mark.parametrize("scheme,alpha", [("euler", 0.5), ("midpoint", 0.5), ("midpoint", 0.25), ("trapezoid", 0.5)])
@pytest.mark.parametrize("bc", [oc.BC_ZERO, oc.BC_PERIODIC])
def test_heat_schemes_eigen_decay(scheme, alpha, bc):
    """One implicit step (tol_abs = 6e-6, implicit.jl:67-70) from an eigenvector IC -- sin(πx)sin(πy)
    for bc_zero!, cos(2πi/N)cos(2πj/N) for bc_periodic! -- reproduces the scheme's exact amplification
    factor with a single Krylov iteration."""
    N = 40
    P = oc.heat2d_euler(N, scheme=scheme, bc=bc, alpha=alpha)
    h = P.hx
    if bc == oc.BC_ZERO:
        u0 = oc.sin_ic(P)
        s2 = math.sin(math.pi * h / 2) ** 2
    else:
        ph = np.cos(2 * np.pi * np.arange(N) / N)
        u0 = np.ascontiguousarray(ph[:, None] * ph[None, :])
        s2 = math.sin(math.pi / N) ** 2
    mu = -P.a * 8.0 / (h * h) * s2
    P.un = u0
    u, st = oc.newton_krylov(P, u0, tol_abs=6e-6)
    assert st["solved"] and st["inner_iterations"] == 1
    assert np.max(np.abs(u - _decay(scheme, P.dt, mu, alpha) * u0)) < 1e-10


def test_heat3d_schemes_periodic_eigen_decay():
    """3D (build-defined) analogue: the periodic cos mode in x, y, z, every scheme."""
    N = 10
    c = np.cos(2 * np.pi * np.arange(N) / N)
    u0 = np.ascontiguousarray(c[:, None, None] * c[None, :, None] * c[None, None, :])
    for scheme in ("euler", "midpoint", "trapezoid"):
        P = oc.heat3d_euler(N, scheme=scheme, bc=oc.BC_PERIODIC, un=u0)
        mu = -P.a * 12.0 / (P.hx * P.hx) * math.sin(math.pi / N) ** 2
        u, st = oc.newton_krylov(P, u0, tol_abs=6e-6)
        assert st["solved"] and st["inner_iterations"] == 1
        assert np.max(np.abs(u - _decay(scheme, P.dt, mu) * u0)) < 1e-10


# ----------------------------------------------------------------------------- preconditioners
def _dense_ilu0(J):
    """Textbook IKJ ILU(0) on J's own sparsity pattern (dense storage, small n)."""
    A = J.copy()
    pat = A != 0
    n = len(A)
    for i in range(n):
        for k in range(i):
            if pat[i, k]:
                A[i, k] = A[i, k] / A[k, k]
                for j in range(k + 1, n):
                    if pat[i, j]:
                        A[i, j] = A[i, j] - A[i, k] * A[k, j]
    return np.tril(A, -1) + np.eye(n), np.triu(A)


@pytest.mark.parametrize("P", [oc.bratu1d(30), oc.bratu2d(7, 5),
                               oc.heat3d_euler(4, 3, 5, un=np.zeros((5, 3, 4)), scheme="midpoint", alpha=0.3),
                               oc.heat2d_euler(6, 4, un=np.zeros((4, 6)), scheme="trapezoid")],
                         ids=["bratu1d", "bratu2d", "heat3d-midpoint", "heat2d-trapezoid"])
def test_ilu0_matches_textbook_ilu0_of_collect(P):
    """oc_ilu0_factor's pivots == the diagonal of a textbook IKJ ILU(0) of collect(J) (bit for bit);
    the two-sweep solve == (LU)^-1 v; for the 1D tridiagonal J, L U == J (the exact LU that
    ilu(collect(J)) is for bratu.jl's 1D problem)."""
    u = oc.sin_ic(P) if P.kind in (oc.BRATU1D, oc.BRATU2D) else np.random.default_rng(0).standard_normal(P.shape)
    n = P.n
    J = np.stack([oc.jv_exact(P, u, np.eye(n)[j].reshape(P.shape)).reshape(-1) for j in range(n)], axis=1)
    L, U = _dense_ilu0(J)
    d = oc.ilu0_factor(P, u).reshape(-1)
    assert np.array_equal(np.diag(U), d)
    v = np.random.default_rng(1).standard_normal(n)
    z = oc.ilu0_solve(P, d, v.reshape(P.shape)).reshape(-1)
    zref = np.linalg.solve(U, np.linalg.solve(L, v))
    assert np.max(np.abs(z - zref)) <= 1e-13 * np.max(np.abs(zref))
    if P.kind == oc.BRATU1D:
        assert np.max(np.abs(L @ U - J)) <= 1e-9 * np.max(np.abs(J))


def test_ilu_preconditioned_newton_bratu1d(golden_dir):
    """bratu.jl:119-137 (GMRES / FGMRES + ilu(collect(J))) at config-1 size: with the exact LU every
    Newton step takes one Krylov iteration; the root is the analytic solution's discretisation
    (bratu.jl:33-37, to the discretisation error like the unpreconditioned solve)."""
    g = np.load(os.path.join(golden_dir, "bratu1d_n1000.npz"))
    P = oc.bratu1d(1000)
    u0 = oc.sin_ic(P)
    for algo in ("gmres", "fgmres"):
        u, st = oc.newton_krylov(P, u0, algo=algo, N="ilu")
        assert st["solved"] and st["inner_iterations"] == st["outer_iterations"]
        assert np.max(np.abs(u - g["true_sol"])) < 3e-4


def test_preconditioned_gmres_restatements():
    """gmres! with N applies N once per cycle (x += N (V y)), fgmres! stores Z_k = N V_k: for a fixed
    diagonal N both give the same residual history; the GMRES preconditioner (bratu.jl:139-157) only
    makes sense flexibly and cuts the outer iterations."""
    P = oc.bratu2d(24, 20)
    u0 = oc.sin_ic(P)
    b = oc.residual(P, u0)
    d = oc.jacobian_diag(P, u0, reciprocal=True)
    kw = dict(restart=True, memory=10, itmax=60, atol=0.0, rtol=1e-10)
    xg, sg, hg = oc.krylov_solve(P, u0, b, algo="gmres", N=("diag", d), **kw)
    xf, sf, hf = oc.krylov_solve(P, u0, b, algo="fgmres", N=("diag", d), **kw)
    assert sg["niter"] == sf["niter"]
    np.testing.assert_allclose(hg[:11], hf[:11], rtol=1e-12)
    assert np.linalg.norm(xg - xf) <= 1e-10 * np.linalg.norm(xf)
    x0, s0, _ = oc.krylov_solve(P, u0, b, **kw)
    x5, s5, _ = oc.krylov_solve(P, u0, b, algo="fgmres", N=("gmres", 5), **kw)
    assert s5["solved"] and s5["niter"] < s0["niter"]
    xs, ss, _ = oc.krylov_solve(P, u0, b, memory=100, itmax=1000, atol=0.0, rtol=1e-13)
    assert ss["solved"] and np.linalg.norm(x5 - xs) <= 1e-8 * np.linalg.norm(xs)


# ----------------------------------------------------------------------------- left preconditioner M
@pytest.mark.parametrize("restart,memory,reorth", [(False, 20, False), (True, 10, False), (True, 8, True)])
def test_left_preconditioned_gmres_c_matches_python(restart, memory, reorth):
    """gmres! with M (src/Ariadne.jl:327-329 forwards M = M(J)): r0 = M b, q = M A V_k, the history is
    the preconditioned residual -- C and numpy restatements agree (Jacobi M)."""
    P = oc.bratu2d(12, 10)
    u = oc.sin_ic(P)
    b = oc.residual(P, u)
    d = oc.jacobian_diag(P, u, reciprocal=True)
    kw = dict(memory=memory, restart=restart, reorthogonalization=reorth, atol=1e-12, rtol=1e-10, itmax=120)
    x_c, st_c, h_c = oc.krylov_solve(P, u, b, M=("diag", d), **kw)
    A = lambda v: oc.jv_exact(P, u, v.reshape(P.shape)).ravel()
    x_p, st_p, h_p = ar.gmres(A, b.ravel(), M=lambda v: d.ravel() * v, **kw)
    assert st_c["niter"] == st_p.niter and st_c["solved"] == st_p.solved
    assert np.allclose(h_c[: memory + 1], h_p[: memory + 1], rtol=1e-8, atol=0)
    assert h_c[0] == pytest.approx(np.linalg.norm(d * b), rel=1e-14)  # beta = ||M b||
    assert _rel(x_c.ravel(), x_p) < 1e-8
    # M only changes the Krylov space: x still solves J x = b
    assert _rel(oc.jv_exact(P, u, x_c).ravel(), b.ravel()) < 1e-7


def test_left_ilu_is_exact_for_bratu1d():
    """For the tridiagonal 1D J, ILU(0) is the exact LU: M = J^-1, so M A = I and left-preconditioned
    GMRES converges in one Arnoldi step to x = J^-1 b (known answer)."""
    P = oc.bratu1d(400)
    u = oc.sin_ic(P)
    b = oc.residual(P, u)
    D = oc.ilu0_factor(P, u)
    x, st, h = oc.krylov_solve(P, u, b, M=("ilu0", D), atol=0.0, rtol=1e-10)
    assert st["solved"] and st["niter"] == 1
    assert _rel(oc.jv_exact(P, u, x), b) < 1e-8
    xn, stn, _ = oc.krylov_solve(P, u, b, N=("ilu0", D), atol=0.0, rtol=1e-10)
    assert stn["niter"] == 1 and _rel(x, xn) < 1e-8


def test_preconditioned_cg_c_matches_python():
    """cg! with M: z = M r, gamma = <r, z>.  The Bratu J is negative definite, so the SPD M is
    -1 ./ diag(J); the Jacobi M cuts the iterations on a variable-diagonal problem."""
    P = oc.bratu1d(300)
    u = 3.0 * oc.sin_ic(P)
    b = oc.residual(P, u)
    m = -oc.jacobian_diag(P, u, reciprocal=True)
    assert np.all(m > 0)
    x_c, st_c, h_c = oc.krylov_solve(P, u, b, algo="cg", atol=1e-12, rtol=1e-10, M=("diag", m))
    A = lambda v: oc.jv_exact(P, u, v)
    x_p, st_p, h_p = ar.cg(A, b.copy(), atol=1e-12, rtol=1e-10, M=lambda v: m * v)
    assert st_c["niter"] == st_p.niter and st_c["solved"]
    np.testing.assert_allclose(h_c[:20], h_p[:20], rtol=1e-8)
    assert _rel(x_c, x_p) < 1e-6
    assert _rel(oc.jv_exact(P, u, x_c), b) < 1e-6


def test_newton_left_preconditioned_bratu1d(golden_dir):
    """newton_krylov!(…; M = ilu) on config 1: every Krylov solve takes one step (M = J^-1)."""
    g = np.load(os.path.join(golden_dir, "bratu1d_n1000.npz"))
    P = oc.bratu1d(1000)
    u, st = oc.newton_krylov(P, oc.sin_ic(P), M="ilu")
    assert st["solved"] and st["inner_iterations"] == st["outer_iterations"]
    assert np.max(np.abs(u - g["true_sol"])) < 3e-4


def test_fd_gmres_sensitivity():
    """Why Bratu FD-GMRES parity is a tolerance, not bits: the oracle against ITSELF.  Changing only the
    summation order of its reductions (chunk 7 instead of 8192) moves a restarted FD-GMRES(10) history
    on 2D Bratu 24^2 by ~1e-9; perturbing F0 = F(u) by at most 1 ulp per element -- what ocml's exp vs
    glibc's does to the GPU's F -- moves it by ~1e-2 where ||r|| > 1e-4 ||r0|| (the FD quotient divides
    the perturbation by eps_fd ~ 1e-8 and the restarts feed it back).  The GPU run of the same solve
    sits at 3.7e-3 (tests/test_hip.py::test_gmres_matches_oracle, tools/fd_probe.py)."""
    P = oc.bratu2d(24)
    u = oc.sin_ic(P)
    b = oc.residual(P, u)
    kw = dict(restart=True, memory=10, atol=1e-12, rtol=1e-9, itmax=150)
    F0p = b + np.random.default_rng(0).choice([-1.0, 0.0, 1.0], b.shape) * np.spacing(np.abs(b))
    try:
        x1, s1, h1 = oc.krylov_solve(P, u, b, jv="fd", F0=b, **kw)
        oc.set_chunk(7)
        x2, s2, h2 = oc.krylov_solve(P, u, b, jv="fd", F0=b, **kw)
    finally:
        oc.set_chunk(8192)
    x3, s3, h3 = oc.krylov_solve(P, u, b, jv="fd", F0=F0p, **kw)
    assert s1["niter"] == s2["niter"] == s3["niter"] == 150
    k = h1 > 1e-4 * h1[0]
    d_order = np.max(np.abs(h2[k] - h1[k]) / h1[k])
    d_ulp = np.max(np.abs(h3[k] - h1[k]) / h1[k])
    assert 0 < d_order < 1e-7, d_order
    assert d_ulp > 1e-4, d_ulp
    np.testing.assert_allclose(h3[:11], h1[:11], rtol=1e-7)  # the first cycle is still tight


def test_bratu_operator_against_the_platform_exp():
    """The shared correctly rounded exp (nk_exp.h, compiled by the HIP stencils AND the oracle) against the
    platform libm's exp (glibc; faithful like Julia's Base.exp, not proven correctly rounded) in the same
    oracle (oracle/_build/libnkoracle_libm.so): a regression in the shared exp cannot hide behind device
    and oracle results that agree because they share it.  Bratu residual, exact JVP and FD operator within
    the ulp bounds one faithful exp allows; exp itself at most 1 ulp apart.  Where glibc (or Base.exp)
    misrounds, the two differ by that ulp: parity against the reference's Base.exp is unpinned there."""
    rng = np.random.default_rng(11)
    P = oc.bratu2d(256, 192)
    u = oc.sin_ic(P) + 0.05 * rng.standard_normal(P.shape)
    v = rng.standard_normal(P.shape)
    ulp = lambda a: np.spacing(np.abs(a))  # noqa: E731
    e_cr, e_lm = oc.exp(u.ravel()), np.exp(u.ravel())  # (numpy's exp: the platform libm too)
    assert np.all(np.abs(e_cr - e_lm) <= ulp(e_cr))
    nl = P.lam * np.exp(u)  # the nonlinear term, where the two exps enter
    F_cr, F_lm = oc.residual(P, u), oc.residual(P, u, libm=True)
    assert np.all(np.abs(F_cr - F_lm) <= 2 * ulp(nl) + ulp(F_cr))
    J_cr, J_lm = oc.jv_exact(P, u, v), oc.jv_exact(P, u, v, libm=True)
    assert np.all(np.abs(J_cr - J_lm) <= 2 * ulp(nl * v) + ulp(J_cr))
    eps = 1e-7
    D_cr, D_lm = oc.jv_fd(P, u, v, eps=eps), oc.jv_fd(P, u, v, eps=eps, libm=True)
    w = u + eps * v
    bound = (2 * ulp(P.lam * np.exp(w)) + ulp(F_cr + eps * v) + 2 * ulp(nl) + ulp(F_cr)) / eps + 2 * ulp(D_cr)
    assert np.all(np.abs(D_cr - D_lm) <= bound)


# ----------------------------------------------------------------------------- device-order reduction trees
def _fma(a, b, c):
    from fractions import Fraction
    return float(Fraction(a) * Fraction(b) + Fraction(c))  # one rounding (int / int true division is exact-rounded)


def _wave(v):
    a = list(v)
    o = 32
    while o:
        a = [a[l] + a[l ^ o] for l in range(64)]
        o >>= 1
    return a[0]


def _block(acc):
    r = _wave(acc[0:64])
    for w in range(1, 4):
        r += _wave(acc[64 * w:64 * w + 64])
    return r


def _ri(parts):
    acc = []
    for t in range(256):
        s = 0.0
        for m in range(t, len(parts), 256):
            s += parts[m]
        acc.append(s)
    return _block(acc)


def test_device_order_trees_match_their_restatement():
    """The oracle's device-order trees (nk_oracle.c OC_DEVRED, the GPU parity checker of
    tests/test_hip_devred.py) against an independent Python restatement of the kernels' summation order:
    64-lane butterfly wave sums, block sums in wave order, reduce_input's thread-strided sums, the chunked
    streaming kernels (k_sumsq / k_mgs_pass / k_update_x), the resident sweep's balanced slot partition and
    polling wave, k_st2d's tiles (256 VEC columns x rows).  Exact equality."""
    rng = np.random.default_rng(11)
    n = 6002  # odd double2 count and a tail-free even n; 3001 double2 elements
    x = rng.standard_normal(n)
    y = rng.standard_normal(n)
    G = 5
    d = oc.dr_trees(n, x, y, G=G, nx=600, ny=10)
    n2 = n // 2
    # chunked: block b owns [b per, (b + 1) per) of the double2 elements, per a multiple of 256
    per = ((n2 + G - 1) // G + 255) // 256 * 256
    chunk = []
    for b in range(G):
        acc = [0.0] * 256
        for i in range(b * per, min((b + 1) * per, n2)):
            t = (i - b * per) % 256
            acc[t] = _fma(x[2 * i], y[2 * i], acc[t])
            acc[t] = _fma(x[2 * i + 1], y[2 * i + 1], acc[t])
        chunk.append(_block(acc))
    assert list(d["chunk"]) == chunk
    assert d["ri_chunk"] == _ri(chunk)
    # the sweep: ceil(n2 / 256) slots, block b owns slots [b S / G, (b + 1) S / G)
    S = (n2 + 255) // 256
    sweep = []
    for b in range(G):
        lo, hi = b * S // G * 256, min((b + 1) * S // G * 256, n2)
        acc = [0.0] * 256
        for i in range(lo, hi):
            t = (i - lo) % 256
            acc[t] = _fma(x[2 * i], y[2 * i], acc[t])
            acc[t] = _fma(x[2 * i + 1], y[2 * i + 1], acc[t])
        sweep.append(_block(acc))
    assert list(d["sweep"]) == sweep
    lanes = []
    for l in range(64):
        p = 0.0
        for j in range(4):
            p += sweep[64 * j + l] if 64 * j + l < G else 0.0
        lanes.append(p)
    assert d["poll1"] == _wave(lanes)
    # k_st2d tiles: 600 x 10 -> 2 tiles of 512 columns, 8-row tiles (the 8-row minimum): 2 x 2 tiles
    nx, ny, rows = 600, 10, 8
    X, Y = x[:nx * ny], y[:nx * ny]
    tiles = []
    for ty in range(2):
        for tx in range(2):
            acc = [0.0] * 256
            for t in range(256):
                x0 = tx * 512 + 2 * t
                if x0 >= nx:
                    continue
                a = 0.0
                for j in range(ty * rows, min(ty * rows + rows, ny)):
                    for k in range(2):
                        a = _fma(X[j * nx + x0 + k], Y[j * nx + x0 + k], a)
                acc[t] = a
            tiles.append(_block(acc))
    assert list(d["tiles"]) == tiles
    assert d["ri_tiles"] == _ri(tiles)
    # k_st3l tiles: 4 rows (one per wave) x 64 VEC columns, z-chunks of 16 planes (blocks; the same here for the
    # single domain: 20 planes x 36 tiles stay under 8192 tiles), thread (wave, lane) upward over its planes
    import ctypes as C
    nx, ny, nz = 130, 9, 20
    X3, Y3 = rng.standard_normal(nx * ny * nz), rng.standard_normal(nx * ny * nz)
    L = oc.lib()
    nt = L.oc_dr_tile_parts3d(nx, ny, nz, 1, oc._p(X3), oc._p(Y3), None)
    got = np.zeros(nt)
    L.oc_dr_tile_parts3d(nx, ny, nz, 1, oc._p(X3), oc._p(Y3), oc._p(got))
    tx_n, ty_n, pl = 2, 3, nx * ny  # 130 columns (VEC 2): 2 tiles of 128 (the second 2 wide); 9 rows: 3 tiles of 4
    want = []
    for tz in range(2):
        for ty in range(ty_n):
            for tx in range(tx_n):
                acc = [0.0] * 256
                for t in range(256):
                    j, x0 = ty * 4 + t // 64, tx * 128 + (t % 64) * 2
                    if x0 >= nx or j >= ny:
                        continue
                    a = 0.0
                    for k in range(tz * 16, min(tz * 16 + 16, nz)):
                        for q in range(2):
                            a = _fma(X3[k * pl + j * nx + x0 + q], Y3[k * pl + j * nx + x0 + q], a)
                    acc[t] = a
                want.append(_block(acc))
    assert nt == len(want) and list(got) == want


def test_device_order_gmres_is_a_reordering_only():
    """Device-order mode changes only the summation order: a restarted FD-GMRES(20) history agrees with the
    default mode to rounding-order differences (and is itself deterministic)."""
    P = oc.bratu2d(128, 96)
    u0 = oc.sin_ic(P)
    F = oc.residual(P, u0)
    kw = dict(jv="fd", F0=F, memory=20, restart=True, atol=0.0, rtol=0.0, itmax=60)
    x0, _, h0 = oc.krylov_solve(P, u0, F, **kw)
    oc.set_devred(True)
    try:
        x1, _, h1 = oc.krylov_solve(P, u0, F, **kw)
        x2, _, h2 = oc.krylov_solve(P, u0, F, **kw)
    finally:
        oc.set_devred(False)
    assert np.array_equal(h1, h2) and np.array_equal(x1, x2)
    assert np.allclose(h1, h0, rtol=1e-7, atol=0)
    assert np.max(np.abs(x1 - x0)) <= 1e-7 * np.max(np.abs(x0))


@pytest.mark.parametrize("algo,side,kind", [("gmres", "N", "diag"), ("fgmres", "N", "diag"), ("gmres", "M", "diag"),
                                            ("gmres", "N", "ilu0"), ("fgmres", "N", "gmres"), ("cg", "M", "negdiag")])
def test_device_order_preconditioned_is_a_reordering_only(algo, side, kind):
    """The preconditioned paths of the device-order mode (||N V_k||, ||M b||, <V_1, M J V_k>, <r, M r> in their
    kernels' trees): the same solve as the default mode up to summation order, and deterministic.  OC_DEV_BNORM
    (the Newton driver's ||F||) is consumed by the outer solve only -- an inner GMRES preconditioner sums its own."""
    P = oc.bratu2d(64, 48)
    u0 = oc.sin_ic(P) + 0.05 * np.random.default_rng(4).standard_normal(P.shape)
    F = oc.residual(P, u0)
    d = oc.jacobian_diag(P, u0, reciprocal=True)
    prec = {"diag": ("diag", d), "negdiag": ("diag", -d), "ilu0": ("ilu0", oc.ilu0_factor(P, u0)), "gmres": ("gmres", 5)}[kind]
    kw = dict(algo=algo, jv="fd", F0=F, memory=20, atol=0.0, rtol=0.0, itmax=40, **{side: prec})
    if algo != "cg":
        kw["restart"] = algo == "gmres"
    x0, s0, h0 = oc.krylov_solve(P, u0, F, **kw)
    oc.set_devred(True)
    try:
        x1, s1, h1 = oc.krylov_solve(P, u0, F, **kw)
        x2, _, h2 = oc.krylov_solve(P, u0, F, **kw)
        un, sn = oc.newton_krylov(P, oc.sin_ic(P), algo="fgmres", N=("gmres", 5), jv="fd", memory=20)
    finally:
        oc.set_devred(False)
    assert np.array_equal(h1, h2) and np.array_equal(x1, x2)
    assert s0["niter"] == s1["niter"] and s0["n_matvec"] == s1["n_matvec"]
    # an inner GMRES is a nonlinear N: FGMRES carries its summation-order differences forward (7e-6 at step 40)
    tol = 1e-4 if kind == "gmres" else 1e-6
    assert np.allclose(h1, h0, rtol=tol, atol=0)
    assert np.max(np.abs(x1 - x0)) <= tol * np.max(np.abs(x0))
    ud, sd = oc.newton_krylov(P, oc.sin_ic(P), algo="fgmres", N=("gmres", 5), jv="fd", memory=20)
    assert sn["solved"] and sd["solved"] and sn["outer_iterations"] == sd["outer_iterations"]
    assert np.max(np.abs(un - ud)) <= 1e-8 * np.max(np.abs(ud))
