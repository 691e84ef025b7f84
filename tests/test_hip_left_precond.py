"""GPU tests of the left preconditioner M (Krylov.jl 0.10's `M`, ldiv = false), which Ariadne forwards
as `M = M(J)` (src/Ariadne.jl:327-329): gmres! / fgmres! take r0 = M (b - A x) and the Arnoldi vector
q = M A (N V_k), and their stopping test measures ||M r||; cg! takes M as its SPD preconditioner
(z = M r, gamma = <r, z>, p = z + beta p).  The oracle restates the same algorithms (C and numpy,
cross-checked in tests/test_oracle.py; Krylov.jl itself is absent: parity against the reference is
unpinned beyond the known answer that ILU(0) of the 1D Jacobian is its exact LU, so M = J^-1 and every
left-preconditioned solve takes one step).  The bar: equal iteration and matvec counts, residual
histories to 1e-8 relative over the first cycle, solutions to the solve's tolerance -- and, against the
oracle in the device's reduction order, histories and solutions bit for bit.
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


def bratu(nx=48, ny=40, seed=4):
    P = oc.bratu2d(nx, ny)
    u0 = oc.sin_ic(P) + 0.05 * np.random.default_rng(seed).standard_normal(P.shape)
    u = ah.DeviceArray.from_numpy(u0)
    res = u.zero()
    p = (P.hx, P.hy, P.lam)
    ah.bratu2d_(res, u, p)
    return P, u0, u, res, p


def devred(fn, *a, **k):
    """An oracle call in the device's reduction order (oracle.set_devred, test_hip_devred.py)."""
    oc.set_devred(True)
    try:
        return fn(*a, **k)
    finally:
        oc.set_devred(False)


def solve(J, b, algo, **kw):
    ws = ah.krylov_workspace(algo, ah.KrylovConstructor(b, memory=kw.pop("memory", 20)))
    ah.krylov_solve_(ws, J, b, history=True, **kw)
    out = (ws.x.to_numpy(), ws.stats)
    ws.free()
    return out


def test_identity_left_preconditioner_matches_unpreconditioned(ctx):
    """M = I through the preconditioned path (a separate dot launch, beta = ||M b|| recomputed): the
    same iterates up to the reduction order."""
    P, u0, u, res, p = bratu()
    J = ah.JacobianOperator(ah.bratu2d_, res, u, p, jv="exact")
    one = u.zero().fill_(1.0)
    kw = dict(restart=True, itmax=60, atol=0.0, rtol=0.0, memory=15)
    x0, s0 = solve(J, res, "gmres", **kw)
    x1, s1 = solve(J, res, "gmres", M=ah.DiagonalPreconditioner(one), **kw)
    assert s0.niter == s1.niter == 60 and s0.n_matvec == s1.n_matvec
    np.testing.assert_allclose(s1.residuals, s0.residuals, rtol=1e-9)
    assert np.linalg.norm(x1 - x0) <= 1e-10 * np.linalg.norm(x0)


@pytest.mark.parametrize("algo", ["gmres", "fgmres"])
@pytest.mark.parametrize("jv", ["exact", "fd"])
def test_jacobi_left_preconditioned_matches_oracle(ctx, algo, jv):
    P, u0, u, res, p = bratu()
    J = ah.JacobianOperator(ah.bratu2d_, res, u, p, jv=jv)
    kw = dict(restart=True, itmax=70, atol=0.0, rtol=1e-10, memory=25)
    x, st = solve(J, res, algo, M=ah.jacobi(J), **kw)
    b = oc.residual(P, u0)
    d = oc.jacobian_diag(P, u0, reciprocal=True)
    xo, so, ho = oc.krylov_solve(P, u0, b, algo=algo, jv=jv, M=("diag", d), **kw)
    assert st.niter == so["niter"] and st.n_matvec == so["n_matvec"]
    assert st.residuals[0] == pytest.approx(np.linalg.norm(d * b), rel=1e-13)  # beta = ||M b||
    np.testing.assert_allclose(st.residuals[:26], ho[:26], rtol=1e-8)
    assert np.linalg.norm(x - xo) <= 1e-6 * np.linalg.norm(xo)
    xr, _, hr = devred(oc.krylov_solve, P, u0, b, algo=algo, jv=jv, M=("diag", d), **kw)  # device order: bitwise
    np.testing.assert_array_equal(np.array(st.residuals), hr)
    np.testing.assert_array_equal(x, xr)


def test_left_and_right_preconditioners_together(ctx):
    """gmres! with both: q = M A N V_k, x += N (V y)."""
    P, u0, u, res, p = bratu(40, 32)
    J = ah.JacobianOperator(ah.bratu2d_, res, u, p, jv="exact")
    kw = dict(restart=True, itmax=60, atol=0.0, rtol=1e-10, memory=20)
    x, st = solve(J, res, "gmres", N=ah.jacobi(J), M=ah.ilu0(J), **kw)
    b = oc.residual(P, u0)
    d = oc.jacobian_diag(P, u0, reciprocal=True)
    D = oc.ilu0_factor(P, u0)
    xo, so, ho = oc.krylov_solve(P, u0, b, N=("diag", d), M=("ilu0", D), **kw)
    assert st.niter == so["niter"] and st.solved == so["solved"]
    np.testing.assert_allclose(st.residuals[:21], ho[:21], rtol=1e-8)
    assert np.linalg.norm(x - xo) <= 1e-6 * np.linalg.norm(xo)
    xr, _, hr = devred(oc.krylov_solve, P, u0, b, N=("diag", d), M=("ilu0", D), **kw)
    np.testing.assert_array_equal(np.array(st.residuals), hr)
    np.testing.assert_array_equal(x, xr)


@pytest.mark.parametrize("algo", ["gmres", "fgmres"])
def test_left_ilu_is_exact_for_bratu1d(ctx, algo):
    """Known answer: ILU(0) of the tridiagonal 1D Jacobian is its exact LU, so M A = I and the solve
    takes one Arnoldi step to x = J^-1 b."""
    P = oc.bratu1d(1000)
    u0 = oc.sin_ic(P)
    u = ah.DeviceArray.from_numpy(u0)
    res = u.zero()
    ah.bratu_(res, u, (P.hx, P.lam))
    J = ah.JacobianOperator(ah.bratu_, res, u, (P.hx, P.lam), jv="exact")
    x, st = solve(J, res, algo, M=ah.ilu0(J), atol=0.0, rtol=1e-10)
    assert st.solved and st.niter == 1
    b = oc.residual(P, u0)
    assert np.linalg.norm(oc.jv_exact(P, u0, x) - b) <= 1e-7 * np.linalg.norm(b)


def test_preconditioned_cg_matches_oracle(ctx):
    """cg! with the SPD M = -1 ./ diag(J) (J is negative definite) on 1D Bratu with a variable
    diagonal: equal iterations, histories to 1e-8 over the first steps."""
    P = oc.bratu1d(300)
    u0 = 3.0 * oc.sin_ic(P)
    u = ah.DeviceArray.from_numpy(u0)
    res = u.zero()
    p = (P.hx, P.lam)
    ah.bratu_(res, u, p)
    J = ah.JacobianOperator(ah.bratu_, res, u, p, jv="exact")
    m = ah.DeviceArray.from_numpy(-ah.jacobian_diag(J, reciprocal=True).to_numpy())
    x, st = solve(J, res, "cg", M=ah.DiagonalPreconditioner(m), atol=1e-12, rtol=1e-10)
    b = oc.residual(P, u0)
    mo = -oc.jacobian_diag(P, u0, reciprocal=True)
    np.testing.assert_array_equal(m.to_numpy(), mo)
    xo, so, ho = oc.krylov_solve(P, u0, b, algo="cg", atol=1e-12, rtol=1e-10, M=("diag", mo))
    assert st.solved and st.niter == so["niter"]
    np.testing.assert_allclose(st.residuals[:20], ho[:20], rtol=1e-8)
    assert np.linalg.norm(x - xo) <= 1e-6 * np.linalg.norm(xo)
    xr, _, hr = devred(oc.krylov_solve, P, u0, b, algo="cg", atol=1e-12, rtol=1e-10, M=("diag", mo))
    np.testing.assert_array_equal(np.array(st.residuals), hr)
    np.testing.assert_array_equal(x, xr)


def test_newton_left_default_atol_stagnates_like_the_oracle(ctx):
    """With Krylov.jl's default atol = √eps the stopping test sees ||M F||: Jacobi's M ~ h²/4 makes it
    fall below atol after a few steps, the solves return x = 0 (niter 0) and Newton stalls -- the
    restated Krylov.jl behaviour, reproduced step for step (same counts, same final ||F||)."""
    P = oc.bratu2d(48, 40)
    u0 = oc.sin_ic(P)
    ref, so = oc.newton_krylov(P, u0, M="jacobi")
    u, r = ah.newton_krylov_(ah.bratu2d_, ah.DeviceArray.from_numpy(u0), (P.hx, P.hy, P.lam), M=ah.jacobi)
    assert not r.solved and not so["solved"]
    assert (r.stats.outer_iterations, r.stats.inner_iterations) == (so["outer_iterations"], so["inner_iterations"])
    assert r.stats.n_res == pytest.approx(so["n_res"], rel=1e-4)  # a stalled iterate: rounding is not damped
    uo, sd = devred(oc.newton_krylov, P, u0, M="jacobi")  # in the device's order: the same bits
    assert r.stats.n_res == sd["n_res"]
    np.testing.assert_array_equal(u.to_numpy(), uo)


@pytest.mark.parametrize("M", ["jacobi", "ilu"])
def test_newton_left_preconditioned_bratu2d_matches_oracle(ctx, M):
    """newton_krylov!(…; M = jacobi / ilu, krylov_kwargs = (; atol = 0)): M(J) is rebuilt every Newton
    step; equal Newton / Krylov / matvec counts with the oracle's driver."""
    P = oc.bratu2d(48, 40)
    u0 = oc.sin_ic(P)
    ref, so = oc.newton_krylov(P, u0, M=M, atol=0.0)
    u, r = ah.newton_krylov_(ah.bratu2d_, ah.DeviceArray.from_numpy(u0), (P.hx, P.hy, P.lam),
                             M=ah.jacobi if M == "jacobi" else ah.ilu0, krylov_kwargs=dict(atol=0.0))
    assert r.solved and so["solved"]
    assert (r.stats.outer_iterations, r.stats.inner_iterations) == (so["outer_iterations"], so["inner_iterations"])
    assert r.n_matvec == so["n_matvec"]
    np.testing.assert_allclose(u.to_numpy(), ref, rtol=0, atol=1e-9 * np.abs(ref).max())
    uo, _ = devred(oc.newton_krylov, P, u0, M=M, atol=0.0)
    np.testing.assert_array_equal(u.to_numpy(), uo)


def test_newton_left_ilu_bratu1d_config1(ctx, golden_dir):
    """BASELINE config 1 with M = ilu: one Krylov step per Newton step, the analytic root."""
    g = np.load(golden_dir + "/bratu1d_n1000.npz")
    P = oc.bratu1d(1000)
    u0 = oc.sin_ic(P)
    u, r = ah.newton_krylov_(ah.bratu_, ah.DeviceArray.from_numpy(u0), (P.hx, P.lam), M=ah.ilu0)
    assert r.solved and r.stats.inner_iterations == r.stats.outer_iterations
    assert np.max(np.abs(u.to_numpy() - g["true_sol"])) < 3e-4


def test_krylov_kwargs_M_wins_over_factory(ctx):
    """(; M = M(J), krylov_kwargs...): an M inside krylov_kwargs overrides the factory (:327-333)."""
    P = oc.bratu2d(32)
    u0 = oc.sin_ic(P)
    calls = []

    def factory(J):
        calls.append(1)
        return ah.jacobi(J)

    one = ah.DeviceArray.from_numpy(np.ones(P.shape))
    u, r = ah.newton_krylov_(ah.bratu2d_, ah.DeviceArray.from_numpy(u0), (P.hx, P.hy, P.lam), M=factory,
                             krylov_kwargs=dict(M=ah.DiagonalPreconditioner(one)))
    assert r.solved and not calls
