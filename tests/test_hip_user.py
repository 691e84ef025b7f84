"""GPU tests of user residuals (kinds NK_USER1D/2D/3D): F!(res, u, p) written by the
caller -- here with torch on the device -- driving the library's device Newton-Krylov.

The user residuals below restate residuals the library also has as built-in kernels, with the
reference's association order, so the parity bar is the built-in kernel's own bar:
  * heat (no transcendental): the user residual, the user-path FD Jv and the exact Jv are
    BIT-IDENTICAL to the built-in kernels (the library evaluates w = u + eps v and the quotient
    (F(w) - F0)/eps exactly as the fused stencil does; torch rounds each op once, no contraction);
  * Bratu: bit-identical as well -- the torch residual takes its exp from ah.exp_ (nk_vexp, the
    built-in stencils' correctly rounded exp, csrc/nk_exp.h);
  * Krylov / Newton on the user path: equal iteration counts, histories to 1e-12 relative /
    1e-14 of ||b|| absolute (only the fixed summation order of the reductions differs from the
    built-in path), and the oracle's root.
"""
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
    import torch  # noqa: F401  (user residuals below are torch code)

    yield c
    c.sync()


def _lap2(P, hx, hy):
    """((e - 2c) + w)/hx^2 + ((n - 2c) + s)/hy^2 on a (ny + 2, nx) view whose first and last rows
    are the ghost rows; x-boundaries zero (bc_zero!, heat_2D.jl:28-38 / bratu.jl:17-18)."""
    import torch
    import torch.nn.functional as tf

    Q = tf.pad(P, (1, 1))  # zero columns left / right
    c = Q[1:-1, 1:-1]
    e, w = Q[1:-1, 2:], Q[1:-1, :-2]
    n, s = Q[2:, 1:-1], Q[:-2, 1:-1]
    # divide by device tensors: ATen turns division by a host scalar into a reciprocal multiply
    hx2 = torch.tensor(hx * hx, dtype=P.dtype, device=P.device)
    hy2 = torch.tensor(hy * hy, dtype=P.dtype, device=P.device)
    return ((e - 2.0 * c) + w) / hx2 + ((n - 2.0 * c) + s) / hy2, c


def _exp(x):
    """exp.(x) through the library's correctly rounded exp (what the built-in Bratu kernel evaluates)"""
    import torch

    x = x.contiguous()
    y = torch.empty_like(x)
    return ah.exp_(y, x)


def torch_bratu2d(res, u, p):
    hx, hy, lam = p
    lsum, c = _lap2(u.torch(ghosts=True), hx, hy)
    res.torch().copy_(lsum + lam * _exp(c))


def torch_bratu2d_tangent(out, u, v, p):
    import torch

    hx, hy, lam = p
    lsum, c = _lap2(v.torch(ghosts=True), hx, hy)
    out.torch().copy_(lsum + lam * (_exp(u.torch()) * c))


def torch_heat2d(res, u, p):
    """G_Euler!(res, uₙ, Δt, diffusion!, du, u, p, t): res = (uₙ + Δt (a lap u)) - u."""
    un, dt, _du, (a, hx, hy, _bc), _t = p
    lsum, c = _lap2(u.torch(ghosts=True), hx, hy)
    res.torch().copy_((un.torch() + dt * (a * lsum)) - c)


def torch_heat2d_tangent(out, u, v, p):
    _un, dt, _du, (a, hx, hy, _bc), _t = p
    lsum, c = _lap2(v.torch(ghosts=True), hx, hy)
    out.torch().copy_(dt * (a * lsum) - c)


USER_BRATU = ah.UserResidual(torch_bratu2d, torch_bratu2d_tangent, name="torch_bratu2d!")
USER_HEAT = ah.UserResidual(torch_heat2d, torch_heat2d_tangent, name="torch_heat2d!")


def bratu_case(nx, ny, seed=3):
    P = oc.bratu2d(nx, ny)
    u0 = oc.sin_ic(P) + 0.05 * np.random.default_rng(seed).standard_normal(P.shape)
    return P, u0, (P.hx, P.hy, P.lam)


def heat_case(ctx, nx, ny, seed=5):
    rng = np.random.default_rng(seed)
    un = rng.standard_normal((ny, nx))
    P = oc.heat2d_euler(nx, ny, un=un)
    u0 = un + 0.01 * rng.standard_normal(un.shape)
    p = (ah.DeviceArray.from_numpy(un), P.dt, None, (P.a, P.hx, P.hy, ah.bc_zero_), 0.0)
    return P, u0, p


@pytest.mark.parametrize("shape", [(64, 64), (130, 37), (1, 5), (6, 1)])
def test_user_heat_residual_and_jv_bit_identical(ctx, shape):
    P, u0, p = heat_case(ctx, *shape)
    u = ah.DeviceArray.from_numpy(u0)
    v = ah.DeviceArray.from_numpy(np.random.default_rng(9).standard_normal(u0.shape))
    r_user, r_blt = u.zero(), u.zero()
    USER_HEAT(r_user, u, p)
    ah.heat2d_euler_(r_blt, u, p)
    np.testing.assert_array_equal(r_user.to_numpy(), r_blt.to_numpy())
    np.testing.assert_array_equal(r_blt.to_numpy(), oc.residual(P, u0))
    for jv in ("exact", "fd"):
        o_user, o_blt = u.zero(), u.zero()
        ah.mul_(o_user, ah.JacobianOperator(USER_HEAT, r_user, u, p, jv=jv), v, eps=1e-7)
        ah.mul_(o_blt, ah.JacobianOperator(ah.heat2d_euler_, r_blt, u, p, jv=jv), v, eps=1e-7)
        np.testing.assert_array_equal(o_user.to_numpy(), o_blt.to_numpy(), err_msg=jv)


def test_user_bratu_residual_and_jv(ctx):
    P, u0, p = bratu_case(96, 80)
    u = ah.DeviceArray.from_numpy(u0)
    vh = np.random.default_rng(4).standard_normal(u0.shape)
    v = ah.DeviceArray.from_numpy(vh)
    res = u.zero()
    n_res = USER_BRATU.residual_norm(res, u, p)
    ref = oc.residual(P, u0)
    np.testing.assert_array_equal(res.to_numpy(), ref)
    assert n_res == pytest.approx(np.linalg.norm(ref), rel=1e-13)
    out = u.zero()
    ah.mul_(out, ah.JacobianOperator(USER_BRATU, res, u, p, jv="exact"), v)
    np.testing.assert_array_equal(out.to_numpy(), oc.jv_exact(P, u0, vh))
    eps = 1e-7
    ah.mul_(out, ah.JacobianOperator(USER_BRATU, res, u, p, jv="fd"), v, eps=eps)
    np.testing.assert_array_equal(out.to_numpy(), oc.jv_fd(P, u0, vh, F0=oc.residual(P, u0), eps=eps))


@pytest.mark.parametrize("jv", ["exact", "fd"])
def test_user_heat_gmres_matches_builtin(ctx, jv):
    P, u0, p = heat_case(ctx, 96, 64, seed=8)
    u = ah.DeviceArray.from_numpy(u0)
    hists, xs = [], []
    for F in (USER_HEAT, ah.heat2d_euler_):
        res = u.zero()
        F(res, u, p)
        ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=8))
        ah.krylov_solve_(ws, ah.JacobianOperator(F, res, u, p, jv=jv), res, restart=True, itmax=40, atol=0.0,
                         rtol=1e-12, history=True)
        hists.append((ws.stats.niter, np.array(ws.stats.residuals)))
        xs.append(ws.x.to_numpy())
        ws.free()
    assert hists[0][0] == hists[1][0]
    # late entries sit ~1e-10 below ||b||: there the two reduction orders show at ~1e-16 of ||b||
    np.testing.assert_allclose(hists[0][1], hists[1][1], rtol=1e-12, atol=1e-14 * hists[1][1][0])
    # the two paths sum their dot partials in different block orders (fused stencil epilogue vs
    # k_user_epi); restarted FD-GMRES amplifies such 1e-16 differences (tests/test_oracle.py::
    # test_fd_gmres_sensitivity), so x agrees to 3e-11 there, to 1e-11 with the exact tangent
    tol = (1e-11, 1e-14) if jv == "exact" else (1e-9, 1e-12)
    np.testing.assert_allclose(xs[0], xs[1], rtol=tol[0], atol=tol[1] * np.abs(xs[1]).max())


def test_user_bratu_newton_matches_oracle(ctx):
    P, _, p = bratu_case(64, 64)
    u0 = oc.sin_ic(P)
    ref, st = oc.newton_krylov(P, u0, jv="fd", memory=20)
    for F in (USER_BRATU, ah.bratu2d_):
        u = ah.DeviceArray.from_numpy(u0)
        u, r = ah.newton_krylov_(F, u, p, jv="fd", memory=20)
        assert r.solved
        assert r.stats.outer_iterations == st["outer_iterations"], F
        got = u.to_numpy()
        assert np.linalg.norm(got - ref) <= 1e-8 * np.linalg.norm(ref), F
        assert r.stats.n_res <= st["tol"]
        oc.set_devred(True, user=F is USER_BRATU)  # each path in its own device order: bit for bit
        try:
            ud, sd = oc.newton_krylov(P, u0, jv="fd", memory=20)
        finally:
            oc.set_devred(False)
        assert r.stats.inner_iterations == sd["inner_iterations"], F
        np.testing.assert_array_equal(got, ud)


def test_user_cg_runs_on_user_operator(ctx):
    """algo=:cg (examples/bratu.jl:59-63) on the user operator: the same iterates as the built-in one."""
    P, u0, p = heat_case(ctx, 48, 40, seed=2)
    u = ah.DeviceArray.from_numpy(u0)
    out = []
    for F in (USER_HEAT, ah.heat2d_euler_):
        res = u.zero()
        F(res, u, p)
        ws = ah.krylov_workspace("cg", ah.KrylovConstructor(res))
        ah.krylov_solve_(ws, ah.JacobianOperator(F, res, u, p, jv="exact"), res, itmax=30, atol=0.0, rtol=1e-10,
                         history=True)
        out.append((ws.stats.niter, np.array(ws.stats.residuals), ws.x.to_numpy()))
        ws.free()
    assert out[0][0] == out[1][0]
    np.testing.assert_allclose(out[0][1], out[1][1], rtol=1e-12, atol=1e-14 * out[1][1][0])


def test_user_callback_error_propagates(ctx):
    def broken(res, u, p):
        raise ValueError("boom")

    F = ah.UserResidual(broken)
    u = ah.DeviceArray.from_numpy(np.ones((8, 8)))
    with pytest.raises(ah.NKError) as ei:
        F(u.zero(), u, None)
    assert isinstance(ei.value.__cause__, ValueError)
    with pytest.raises(ValueError, match="jv='fd'"):
        ah.JacobianOperator(F, u.zero(), u, None, jv="exact")
