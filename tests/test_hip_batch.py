"""GPU tests of the batched Jacobian-vector products and the device assembly of collect(J).

mul!(Out::AbstractMatrix, J, V) (src/Ariadne.jl:67-84) and its transpose (:109-138) run as ONE
fused launch per 8 columns (nk_jv_batched: u, F(u), u_n read once).  Every column must equal the
single-vector product bit for bit (same operands, same association order) -- for every problem
kind, both boundary conditions, exact and FD, and batch widths that cross the 8-column chunking.
collect(J) (:140-162) is assembled on the device from 2 dim + 1 coloured probes; it must equal
unit-vector probing (the reference's loop) bit for bit, and at 4096^2 (BASELINE config 2) its
diagonal must equal nk_jacobian_diag's and its off-diagonals 1/h^2 exactly.
"""
import numpy as np
import pytest

import _nkpath  # noqa: F401
import ariadne_hip as ah
from oracle import oracle as oc

from test_hip_schemes import device_residual

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = ah.Context(0)
    ah.set_default_context(c)
    yield c
    c.sync()


def problems():
    rng = np.random.default_rng(11)
    out = []
    P = oc.bratu1d(300)
    out.append(pytest.param(P, oc.sin_ic(P), id="bratu1d"))
    P = oc.bratu2d(130, 67)
    out.append(pytest.param(P, oc.sin_ic(P) + 0.1 * rng.standard_normal(P.shape), id="bratu2d"))
    for scheme in ("euler", "midpoint", "trapezoid"):
        for bc in (oc.BC_ZERO, oc.BC_PERIODIC):
            for shape in ((129, 10), (33, 17, 9)):
                un = rng.standard_normal(shape[::-1])
                mk = oc.heat2d_euler if len(shape) == 2 else oc.heat3d_euler
                Q = mk(*shape, un=un, scheme=scheme, bc=bc, alpha=0.3 if scheme == "midpoint" else 0.5)
                out.append(pytest.param(Q, un + 0.01 * rng.standard_normal(un.shape),
                                        id=f"heat{len(shape)}d-{scheme}-bc{bc}"))
    return out


def residual_of(P):
    if P.kind == oc.BRATU1D:
        return ah.bratu_, (P.hx, P.lam)
    if P.kind == oc.BRATU2D:
        return ah.bratu2d_, (P.hx, P.hy, P.lam)
    return device_residual(P)


@pytest.mark.parametrize("jv", ["exact", "fd"])
@pytest.mark.parametrize("P,u0", problems())
def test_batched_columns_equal_single_products(ctx, P, u0, jv):
    F, p = residual_of(P)
    u = ah.DeviceArray.from_numpy(u0)
    res = u.zero()
    F(res, u, p)
    J = ah.JacobianOperator(F, res, u, p, jv=jv)
    rng = np.random.default_rng(3)
    k = 11  # two launches: 8 + 3 columns
    vs = [ah.DeviceArray.from_numpy(rng.standard_normal(P.shape)) for _ in range(k)]
    vs[4].fill_(0.0)  # a zero column (FD: nk_jv's special case)
    outs = [u.zero() for _ in range(k)]
    ctx.prof_reset()
    ctx.prof_enable(1 << 20)
    ah.mul_(outs, J, vs)
    launches = ctx.prof_read().get(f"jv_{jv}_batch", {}).get("launches", 0)
    ctx.prof_enable(0)
    assert launches == 2, "the fused batched kernel did not run"
    single = u.zero()
    for o, v in zip(outs, vs):
        ah.mul_(single, J, v)
        np.testing.assert_array_equal(o.to_numpy(), single.to_numpy())
    if jv == "exact":  # transpose: J^T = J for the built-in stencils
        touts = [u.zero() for _ in range(3)]
        ah.mul_(touts, ah.transpose(J), vs[:3])
        for o, t in zip(outs[:3], touts):
            np.testing.assert_array_equal(o.to_numpy(), t.to_numpy())


@pytest.mark.parametrize("P,u0", [pytest.param(*p.values, id=p.id) for p in problems()
                                  if p.values[0].n <= 4096])
def test_device_collect_equals_unit_probing(ctx, P, u0):
    F, p = residual_of(P)
    u = ah.DeviceArray.from_numpy(u0)
    J = ah.JacobianOperator(F, u.zero(), u, p)
    A = ah.collect(J)
    B = ah.collect(J, coloring="dense")
    assert A.nnz == B.nnz
    np.testing.assert_array_equal(A.toarray(), B.toarray())
    np.testing.assert_array_equal(A.indptr, B.indptr)
    np.testing.assert_array_equal(A.indices, B.indices)  # rows sorted within each column, like SparseMatrixCSC
    np.testing.assert_array_equal(ah.collect(J.T).toarray(), A.T.toarray())


def test_device_collect_bratu2d_4096(ctx):
    """BASELINE config 2's Jacobian (16.8 M rows, 84 M entries) in one batched probe launch."""
    P = oc.bratu2d(4096)
    u0 = oc.sin_ic(P)
    u = ah.DeviceArray.from_numpy(u0)
    J = ah.JacobianOperator(ah.bratu2d_, u.zero(), u, (P.hx, P.hy, P.lam))
    A = ah.collect(J)
    n = P.n
    assert A.shape == (n, n) and A.nnz == 5 * n - 4 * 4096
    d = ah.jacobian_diag(J).to_numpy().reshape(-1)
    np.testing.assert_array_equal(A.diagonal(), d)
    import scipy.sparse as sp

    off = sp.triu(A, 1) + sp.tril(A, -1)
    assert off.nnz == 4 * n - 4 * 4096
    np.testing.assert_array_equal(np.unique(off.data), np.unique([1.0 / (P.hx * P.hx), 1.0 / (P.hy * P.hy)]))
