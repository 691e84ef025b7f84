"""GPU tests of the Krylov / Newton edge cases Krylov.jl 0.10 and Ariadne define (restated in the
oracle: SURVEY.md Appendix A, `src/Ariadne.jl:290-372`): a zero right-hand side (x = 0, no iteration,
solved), an iteration cap below convergence (stopped at itmax, not solved), GMRES's breakdown on a
grid smaller than its memory (the Krylov space exhausted: the exact solution), and a Newton start that
is already a root (no Newton step).  Flags and counts equal the oracle's; histories to 1e-9 relative;
solutions to the tolerance stated per test.  Plus an oracle-independent check: one implicit heat step
of every scheme, 2D and 3D, against scipy's sparse LU of the same linear system."""
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


def setup(P, u0):
    u = ah.DeviceArray.from_numpy(u0)
    res = u.zero()
    if P.kind == oc.BRATU1D:
        F, p = ah.bratu_, (P.hx, P.lam)
    else:
        F, p = ah.bratu2d_, (P.hx, P.hy, P.lam)
    F(res, u, p)
    return ah.JacobianOperator(F, res, u, p, jv="exact"), res


def solve(ws, J, b, **kw):
    ah.krylov_solve_(ws, J, b, history=True, **kw)
    return ws.x.to_numpy(), ws.stats


@pytest.mark.parametrize("algo", ["gmres", "fgmres", "cg"])
def test_zero_rhs(ctx, algo):
    """Krylov.jl: b = 0 -> x = 0 is a zero-residual solution: niter = 0, solved, no matvec, history
    [0] -- and the workspace's x from an earlier solve is overwritten with zeros."""
    P = oc.bratu1d(300) if algo == "cg" else oc.bratu2d(33, 20)
    u0 = oc.sin_ic(P)
    J, res = setup(P, u0)
    ws = ah.krylov_workspace(algo, ah.KrylovConstructor(res, memory=10))
    solve(ws, J, res, itmax=5, atol=0.0, rtol=0.0)  # leaves a non-zero x behind
    assert np.any(ws.x.to_numpy() != 0.0)
    x, st = solve(ws, J, res.zero(), itmax=50)
    xo, so, ho = oc.krylov_solve(P, u0, np.zeros(P.shape), algo=algo, jv="exact", memory=10, itmax=50)
    assert st.niter == so["niter"] == 0 and st.solved and so["solved"]
    assert st.n_matvec == so["n_matvec"] == 0
    assert st.residuals == list(ho) == [0.0]
    assert not np.any(x) and not np.any(xo)


@pytest.mark.parametrize("algo", ["gmres", "fgmres", "cg"])
def test_itmax_cap(ctx, algo):
    """An unreachable tolerance: the solve stops after itmax iterations, not solved, status
    'maximum number of iterations exceeded' -- the oracle's counts, its history to 1e-9."""
    P = oc.bratu1d(300) if algo == "cg" else oc.bratu2d(48, 40)
    u0 = oc.sin_ic(P)
    J, res = setup(P, u0)
    kw = dict(itmax=7, atol=1e-300, rtol=1e-15)
    if algo != "cg":
        kw["restart"] = True
    ws = ah.krylov_workspace(algo, ah.KrylovConstructor(res, memory=5))
    x, st = solve(ws, J, res, **kw)
    xo, so, ho = oc.krylov_solve(P, u0, res.to_numpy(), algo=algo, jv="exact", memory=5, **kw)
    assert st.niter == so["niter"] == 7 and not st.solved and not so["solved"]
    assert st.status == "maximum number of iterations exceeded"
    assert st.n_matvec == so["n_matvec"]
    np.testing.assert_allclose(st.residuals, ho, rtol=1e-9)
    assert np.linalg.norm(x - xo) <= 1e-9 * np.linalg.norm(xo)
    oc.set_devred(True)
    try:
        xr, _, hr = oc.krylov_solve(P, u0, res.to_numpy(), algo=algo, jv="exact", memory=5, **kw)
    finally:
        oc.set_devred(False)
    np.testing.assert_array_equal(np.array(st.residuals), hr)
    np.testing.assert_array_equal(x, xr)


@pytest.mark.parametrize("nx,ny", [(3, 3), (5, 2), (4, 4)])
def test_gmres_exhausts_krylov_space(ctx, nx, ny):
    """GMRES with memory > n and no tolerance: the Arnoldi process runs out of directions (h_{k+1,k}
    at the rounding level -> Krylov.jl's breakdown exit) within n steps; the iterate is the exact
    solution of the dense system, and the step count and flags are the oracle's."""
    P = oc.bratu2d(nx, ny)
    u0 = oc.sin_ic(P) + 0.1
    J, res = setup(P, u0)
    n = nx * ny
    ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=20))
    x, st = solve(ws, J, res, itmax=40, atol=0.0, rtol=0.0)
    xo, so, ho = oc.krylov_solve(P, u0, res.to_numpy(), jv="exact", memory=20, itmax=40, atol=0.0, rtol=0.0)
    assert st.niter == so["niter"] <= n and st.solved == so["solved"]
    assert so["breakdown"] and st.status == "breakdown"
    Jd = np.column_stack([oc.jv_exact(P, u0, e.reshape(P.shape)).reshape(-1) for e in np.eye(n)])
    exact = np.linalg.solve(Jd, res.to_numpy().reshape(-1))
    assert np.max(np.abs(x.reshape(-1) - exact)) <= 1e-10 * np.max(np.abs(exact))
    assert np.max(np.abs(x - xo)) <= 1e-10 * np.max(np.abs(xo))


def test_newton_start_at_root(ctx):
    """newton_krylov! from a root (implicit Euler on a zero field: F(0) = 0): the loop's first check
    ||F|| <= tol holds, no Newton step is taken -- as in the oracle."""
    n = 32
    P = oc.heat2d_euler(n, un=np.zeros((n, n)))
    u0 = np.zeros((n, n))
    ref, so = oc.newton_krylov(P, u0)
    un = ah.DeviceArray.from_numpy(P.un)
    u, r = ah.newton_krylov_(ah.heat2d_euler_, ah.DeviceArray.from_numpy(u0),
                             (un, P.dt, None, (P.a, P.hx, P.hy, ah.bc_zero_), 0.0))
    assert r.solved and so["solved"]
    assert r.stats.outer_iterations == so["outer_iterations"] == 0
    assert r.stats.inner_iterations == so["inner_iterations"] == 0
    assert not np.any(u.to_numpy()) and not np.any(ref)


# ----------------------------------------------------------------------------- direct-solve oracle
def _lap(shape, hs, periodic=False):
    """The Laplacian of a C-ordered (z,) y, x grid as a scipy sparse matrix (x fastest): zero Dirichlet
    (bc_zero!) or wrapped (bc_periodic!, heat_2D.jl:15-26)."""
    import scipy.sparse as sp

    def d1(n, h):
        m = sp.diags([np.ones(n - 1), -2.0 * np.ones(n), np.ones(n - 1)], [-1, 0, 1]).tolil()
        if periodic:
            m[0, n - 1] += 1.0
            m[n - 1, 0] += 1.0
        return m.tocsr() / (h * h)

    L = None
    for n, h in zip(shape, hs):  # slowest axis first: kronsum(A, B) = A (x) I + I (x) B, B the faster axis
        L = d1(n, h) if L is None else sp.kronsum(d1(n, h), L)
    return L.tocsc()


@pytest.mark.parametrize("bc", ["zero", "periodic"])
@pytest.mark.parametrize("dim,scheme", [(2, "euler"), (2, "midpoint"), (2, "trapezoid"), (3, "euler"),
                                        (3, "midpoint"), (3, "trapezoid")])
def test_implicit_step_matches_direct_solve(ctx, dim, scheme, bc):
    """One implicit time step (implicit.jl:8-37: G_Euler!, G_Midpoint! with alpha 0.3, G_Trapezoid!;
    bc_zero! and bc_periodic!)
    is a linear solve -- (I - dt a c L) u = u_n + dt a d L u_n with (c, d) = (1, 0), (1 - alpha, alpha),
    (1/2, 1/2) -- so scipy's sparse LU gives the exact step independently of the oracle: the device
    Newton-Krylov step, solved to ||G|| <= 1e-11, agrees to 1e-10 of max |u|."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as spla

    rng = np.random.default_rng(21)
    alpha = 0.3
    per = bc == "periodic"
    obc, dbc = (oc.BC_PERIODIC, ah.bc_periodic_) if per else (oc.BC_ZERO, ah.bc_zero_)
    if dim == 2:
        n = 160
        un = rng.standard_normal((n, n))
        P = oc.heat2d_euler(n, un=un, scheme=scheme, alpha=alpha, bc=obc)
        hs, diff, bcp = (P.hy, P.hx), ah.diffusion_, (P.a, P.hx, P.hy, dbc)
    else:
        n = 28  # scipy's LU of a 3D 7-point matrix fills in: 28^3 takes ~1 s, 36^3 ~7 s
        un = rng.standard_normal((n, n, n))
        P = oc.heat3d_euler(n, un=un, scheme=scheme, alpha=alpha, bc=obc)
        hs, diff, bcp = (P.hz, P.hy, P.hx), ah.diffusion3d_, (P.a, P.hx, P.hy, P.hz, dbc)
    c, d = {"euler": (1.0, 0.0), "midpoint": (1.0 - alpha, alpha), "trapezoid": (0.5, 0.5)}[scheme]
    L = _lap(un.shape, hs, per)
    A = sp.identity(un.size, format="csc") - (P.dt * P.a * c) * L
    rhs = un.ravel() + (P.dt * P.a * d) * (L @ un.ravel())
    exact = spla.spsolve(A, rhs).reshape(un.shape)
    G = {"euler": ah.G_Euler_, "midpoint": ah.G_Midpoint_(alpha=alpha), "trapezoid": ah.G_Trapezoid_}[scheme]
    F = G.bind(diff)
    und = ah.DeviceArray.from_numpy(un)
    u, r = ah.newton_krylov_(F, und.copy(), (und, P.dt, None, bcp, 0.0), tol_abs=1e-11, tol_rel=0.0,
                             krylov_kwargs={"atol": 1e-15})
    assert r.solved
    assert np.max(np.abs(u.to_numpy() - exact)) <= 1e-10 * np.max(np.abs(exact))
