"""GPU tests of right preconditioning: FGMRES / preconditioned GMRES
in the flexible form, the device Jacobi preconditioner, user preconditioners, and N factories in
newton_krylov_.  Krylov.jl's preconditioned iterates are not pinned by the reference (parity
unpinned), so the bar is: identity-preconditioned == unpreconditioned bit for bit (exact Jv),
jacobian_diag == diag(collect(J)) bit for bit, the preconditioned solves reach the requested
residual (checked with an independent Jv) and the oracle's solution / Newton root.
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


def bratu(nx=72, ny=56, seed=4):
    P = oc.bratu2d(nx, ny)
    u0 = oc.sin_ic(P) + 0.05 * np.random.default_rng(seed).standard_normal(P.shape)
    u = ah.DeviceArray.from_numpy(u0)
    res = u.zero()
    p = (P.hx, P.hy, P.lam)
    ah.bratu2d_(res, u, p)
    return P, u0, u, res, p


def solve(J, b, algo, N=None, **kw):
    ws = ah.krylov_workspace(algo, ah.KrylovConstructor(b, memory=kw.pop("memory", 20)))
    ah.krylov_solve_(ws, J, b, N=N, history=True, **kw)
    out = (ws.x.to_numpy(), ws.stats)
    ws.free()
    return out


def test_jacobian_diag_is_diag_of_collect(ctx):
    P, u0, u, res, p = bratu(17, 13)
    J = ah.JacobianOperator(ah.bratu2d_, res, u, p)
    d = ah.jacobian_diag(J).to_numpy().reshape(-1)
    np.testing.assert_array_equal(d, ah.collect(J).diagonal())
    np.testing.assert_array_equal(ah.jacobian_diag(J, reciprocal=True).to_numpy().reshape(-1), 1.0 / d)


@pytest.mark.parametrize("algo", ["gmres", "fgmres"])
def test_identity_preconditioner_is_bitwise_unpreconditioned(ctx, algo):
    P, u0, u, res, p = bratu()
    J = ah.JacobianOperator(ah.bratu2d_, res, u, p, jv="exact")
    one = u.zero().fill_(1.0)
    x0, s0 = solve(J, res, "gmres", restart=True, itmax=60, atol=0.0, rtol=0.0, memory=15)
    x1, s1 = solve(J, res, algo, N=ah.DiagonalPreconditioner(one), restart=True, itmax=60, atol=0.0, rtol=0.0,
                   memory=15)
    assert s0.niter == s1.niter == 60
    assert s0.residuals == s1.residuals
    np.testing.assert_array_equal(x0, x1)


@pytest.mark.parametrize("jv", ["exact", "fd"])
def test_jacobi_preconditioned_solve_reaches_tolerance(ctx, jv):
    P, u0, u, res, p = bratu()
    J = ah.JacobianOperator(ah.bratu2d_, res, u, p, jv=jv)
    x, st = solve(J, res, "fgmres", N=ah.jacobi(J), restart=True, itmax=2000, atol=0.0, rtol=1e-9, memory=30)
    assert st.solved
    # the true residual, with an independent exact Jv
    Jx = oc.jv_exact(P, u0, x)
    b = oc.residual(P, u0)
    assert np.linalg.norm(b - Jx) <= 1e-7 * np.linalg.norm(b)
    xo, so, _ = oc.krylov_solve(P, u0, b, jv="exact", memory=30, restart=True, itmax=4000, atol=0.0, rtol=1e-11)
    assert np.linalg.norm(x - xo) <= 1e-5 * np.linalg.norm(xo)


def test_user_preconditioner_matches_diagonal(ctx):
    import torch  # noqa: F401

    P, u0, u, res, p = bratu(40, 32)
    J = ah.JacobianOperator(ah.bratu2d_, res, u, p)
    dinv = ah.jacobian_diag(J, reciprocal=True)

    def apply(z, v):
        z.torch().copy_(dinv.torch() * v.torch())

    a = solve(J, res, "gmres", N=ah.jacobi(J), restart=True, itmax=50, atol=0.0, rtol=0.0)
    b = solve(J, res, "gmres", N=ah.UserPreconditioner(apply, u.grid, u.ctx), restart=True, itmax=50, atol=0.0,
              rtol=0.0)
    assert a[1].residuals == b[1].residuals
    np.testing.assert_array_equal(a[0], b[0])


def test_newton_with_jacobi_factory(ctx):
    P = oc.bratu2d(64)
    u0 = oc.sin_ic(P)
    ref, st = oc.newton_krylov(P, u0, memory=20)
    u, r = ah.newton_krylov_(ah.bratu2d_, ah.DeviceArray.from_numpy(u0), (P.hx, P.hy, P.lam), N=ah.jacobi,
                             algo="fgmres", memory=20)
    assert r.solved
    np.testing.assert_allclose(u.to_numpy(), ref, rtol=0, atol=1e-6 * np.abs(ref).max())
    with pytest.raises(ah.NKError):  # CG takes no right preconditioner
        ws = ah.krylov_workspace("cg", ah.KrylovConstructor(u.zero()))
        J = ah.JacobianOperator(ah.bratu2d_, u.zero(), u, (P.hx, P.hy, P.lam))
        ah.krylov_solve_(ws, J, u, N=ah.jacobi(J))
