"""GPU tests of the operator API around mul!: transpose(J) (src/Ariadne.jl:87-107), the batched
form (:59-85), collect(J) (:140-162) -- pinned by the reference's own known answers
(test/runtests.jl:4-54, run through a user residual on the device) and by the oracle.

Tolerances: every entry bit-identical -- heat has no transcendental, and the Bratu kernels and the
Kelley user residual take exp from the correctly rounded nk_exp (csrc/nk_exp.h, shared with the
oracle); colour-probed and unit-probed collect(J) are bit-identical (every probe entry is one
Jacobian entry computed from the same operands).
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


def oracle_dense_jacobian(P, u):
    n = P.n
    J = np.zeros((n, n))
    for j in range(n):
        e = np.zeros(n)
        e[j] = 1.0
        J[:, j] = oc.jv_exact(P, u, e.reshape(P.shape)).reshape(-1)
    return J


@pytest.mark.parametrize("kind", ["bratu1d", "bratu2d", "heat2d", "heat3d"])
def test_collect_matches_oracle_and_unit_probing(ctx, kind):
    rng = np.random.default_rng(5)
    if kind == "bratu1d":
        P = oc.bratu1d(17)
        u0 = oc.sin_ic(P)
        F, p = ah.bratu_, (P.hx, P.lam)
    elif kind == "bratu2d":
        P = oc.bratu2d(9, 7)
        u0 = oc.sin_ic(P) + 0.1 * rng.standard_normal(P.shape)
        F, p = ah.bratu2d_, (P.hx, P.hy, P.lam)
    elif kind == "heat2d":
        un = rng.standard_normal((6, 11))
        P = oc.heat2d_euler(11, 6, un=un)
        u0 = un.copy()
        F, p = ah.heat2d_euler_, (ah.DeviceArray.from_numpy(un), P.dt, None, (P.a, P.hx, P.hy, ah.bc_zero_), 0.0)
    else:
        un = rng.standard_normal((4, 5, 6))
        P = oc.heat3d_euler(6, 5, 4, un=un)
        u0 = un.copy()
        F, p = ah.heat3d_euler_, (ah.DeviceArray.from_numpy(un), P.dt, None, (P.a, P.hx, P.hy, P.hz, ah.bc_zero_), 0.0)
    u = ah.DeviceArray.from_numpy(u0)
    res = u.zero()
    J = ah.JacobianOperator(F, res, u, p)
    A = ah.collect(J).toarray()
    B = ah.collect(J, coloring="dense").toarray()
    np.testing.assert_array_equal(A, B)
    ref = oracle_dense_jacobian(P, u0)
    assert np.array_equal(A != 0, ref != 0)  # the stencil pattern
    np.testing.assert_array_equal(A, ref)
    # transpose: collect(transpose(J)) == transpose(collect(J))  (runtests.jl:54)
    np.testing.assert_array_equal(ah.collect(ah.transpose(J)).toarray(), A.T)


def test_transpose_and_batched_mul(ctx):
    P = oc.bratu2d(40, 33)
    u0 = oc.sin_ic(P)
    u = ah.DeviceArray.from_numpy(u0)
    res = u.zero()
    J = ah.JacobianOperator(ah.bratu2d_, res, u, (P.hx, P.hy, P.lam))
    rng = np.random.default_rng(0)
    vs = [ah.DeviceArray.from_numpy(rng.standard_normal(P.shape)) for _ in range(3)]
    outs = [u.zero() for _ in vs]
    ah.mul_(outs, J, vs)  # batched
    for o, v in zip(outs, vs):
        single = u.zero()
        ah.mul_(single, J, v)
        np.testing.assert_array_equal(o.to_numpy(), single.to_numpy())
        t = u.zero()
        ah.mul_(t, J.T, v)  # symmetric Jacobian
        np.testing.assert_array_equal(t.to_numpy(), single.to_numpy())
    assert J.T.size == tuple(reversed(J.size))


def _exp1m(X):
    """exp(x1 - 1) through the library's correctly rounded exp (ah.exp_, nk_vexp), a 1-element tensor"""
    import torch

    t = (X[0:1] - 1).contiguous()
    return ah.exp_(torch.empty_like(t), t)


def kelley_oop(x, p):
    """runtests.jl:10-14's out-of-place F(x, p) (a new array; x is a torch view of the device vector)"""
    import torch

    return torch.cat([x[0:1] ** 2 + x[1:2] ** 2 - 2, _exp1m(x) + x[1:2] ** 2 - 2])


def _kelley_user():
    """runtests.jl's 2x2 problem, F(x) = [x1^2 + x2^2 - 2, exp(x1 - 1) + x2^2 - 2] (runtests.jl:4-7), as a
    device user residual (torch) with exp from ah.exp_, its tangent -- Enzyme's forward mode of F!, term
    by term -- and transpose tangent."""

    def F(res, x, p):
        X = x.torch()
        r = res.torch()
        r[0] = X[0] ** 2 + X[1] ** 2 - 2
        r[1] = _exp1m(X)[0] + X[1] ** 2 - 2

    def J(out, x, v, p):
        X, V, o = x.torch(), v.torch(), out.torch()
        o[0] = 2 * X[0] * V[0] + 2 * X[1] * V[1]
        o[1] = _exp1m(X)[0] * V[0] + 2 * X[1] * V[1]

    def JT(out, x, w, p):
        X, W, o = x.torch(), w.torch(), out.torch()
        o[0] = 2 * X[0] * W[0] + _exp1m(X)[0] * W[1]
        o[1] = 2 * X[1] * W[0] + 2 * X[1] * W[1]

    return ah.UserResidual(F, J, name="kelley!", JT=JT)


def test_reference_known_answers_through_the_device(ctx, golden_dir):
    with open(os.path.join(golden_dir, "kelley2x2.json")) as f:
        ka = json.load(f)
    K = _kelley_user()
    x = ah.DeviceArray.from_numpy(np.array(ka["x_jvp"]))
    res = x.zero()
    J = ah.JacobianOperator(K, res, x, None)
    out = x.zero()
    ah.mul_(out, J, ah.DeviceArray.from_numpy(np.array([1.0, 0.0])))  # runtests.jl:36-38
    assert out.to_numpy().tolist() == ka["jvp_e1"] == [6.0, 7.38905609893065]  # exactly: exp(2.0), rounded once
    ah.mul_(out, J.T, ah.DeviceArray.from_numpy(np.array([1.0, 0.0])))  # runtests.jl:40-42
    assert out.to_numpy().tolist() == ka["vjp_e1"]
    A = ah.collect(J).toarray()  # runtests.jl:44-46: collect(J) == J_Enz
    assert A.tolist() == ka["jacobian"]
    np.testing.assert_array_equal(ah.collect(J.T).toarray(), A.T)  # runtests.jl:54
    # runtests.jl:57-66 (batched): mul!(Out, J, I) == J_Enz, mul!(Out, transpose(J), I) == collect(transpose(J))
    cols = [ah.DeviceArray.from_numpy(np.array(c)) for c in ([1.0, 0.0], [0.0, 1.0])]
    outs = [x.zero(), x.zero()]
    ah.mul_(outs, J, cols)
    assert np.column_stack([o.to_numpy() for o in outs]).tolist() == ka["jacobian"]
    ah.mul_(outs, J.T, cols)
    np.testing.assert_array_equal(np.column_stack([o.to_numpy() for o in outs]), ah.collect(J.T).toarray())
    for x0 in ka["starts_inplace"]:  # runtests.jl:15-18: newton_krylov! from (2, 0.5) is solved
        u, r = ah.newton_krylov_(K, ah.DeviceArray.from_numpy(np.array(x0)), None)
        assert r.solved
        np.testing.assert_allclose(u.to_numpy(), ka["root"], atol=1e-5)
        u, r = ah.newton_krylov_(K, ah.DeviceArray.from_numpy(np.array(x0)), None, jv="fd")
        assert r.solved
    for x0 in ka["starts_outofplace"]:  # runtests.jl:20-23: newton_krylov(F, (3, 5)) -- out of place -- is solved
        x0d = ah.DeviceArray.from_numpy(np.array(x0))
        u, r = ah.newton_krylov(kelley_oop, x0d, None, jv="fd")
        assert r.solved and x0d.to_numpy().tolist() == x0  # u0 untouched
        # runtests.jl asserts `solved` only: F has two roots (x1^2 = exp(x1 - 1): x1 = 1 or -0.4777...), and
        # from (3, 5) Newton ends at (-0.4777, 1.3311) -- the numpy restatement's root, too
        from oracle import ariadne_ref as ar

        def kelley_np(x, p):  # dual-number aware (ar.dexp): the restatement's forward-mode tangent
            res = np.zeros(2, dtype=object) if x.dtype == object else np.zeros(2)
            res[0] = x[0] ** 2 + x[1] ** 2 - 2
            res[1] = ar.dexp(x[0] - 1) + x[1] ** 2 - 2
            return res

        uo, sto = ar.newton_krylov(kelley_np, np.array(x0))
        assert sto["solved"]
        np.testing.assert_allclose(u.to_numpy(), uo, rtol=1e-8)
        u, r = ah.newton_krylov(K, x0d, None)  # the same start with the exact tangent
        assert r.solved


@pytest.mark.parametrize("reorth", [False, True])
def test_mgs_step_matches_numpy(reorth):
    """nk_mgs_step (the fused MGS sweep as a primitive) against a numpy MGS with Krylov.jl's
    order: h_i = <V_i, q>, q -= h_i V_i (fma), then ||q||; reorthogonalization adds a second sweep."""
    ctx = ah.Context(0)
    ah.set_default_context(ctx)
    rng = np.random.default_rng(4)
    n, k = 5000, 6
    Q, _ = np.linalg.qr(rng.standard_normal((n, k)))
    q0 = rng.standard_normal(n)
    g = ah.Grid.full(n)
    V = [ah.DeviceArray.from_numpy(np.ascontiguousarray(Q[:, i]), g) for i in range(k)]
    qd = ah.DeviceArray.from_numpy(q0, g)
    h = ah.mgs_step_(V, qd, reorthogonalization=reorth)
    q = q0.copy()
    href = np.zeros(k + 1)
    for _ in range(2 if reorth else 1):
        for i in range(k):
            hi = float(np.dot(Q[:, i], q))
            href[i] += hi
            q = q - hi * Q[:, i]
    href[k] = np.linalg.norm(q)
    np.testing.assert_allclose(h, href, rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(qd.to_numpy(), q, rtol=0, atol=1e-13)
