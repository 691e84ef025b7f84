"""GPU parity of the implicit.jl time-stepping schemes and bc_periodic!.

G_Euler! / G_Midpoint!(α) / G_Trapezoid! composed with diffusion! under bc_zero! and bc_periodic!
(examples/implicit.jl:8-37, examples/heat_2D.jl:15-62), 2D and the build-defined 3D analogue, all
through libnkhip.so's C ABI against the C oracle (itself pinned bit for bit to a literal halo-array
restatement of the reference, tests/test_oracle.py).

Tolerances: no transcendental on these paths, both sides compile with -ffp-contract=off and use the
reference's association order -> residual, exact JVP, FD JVP and diag(J) are bit-identical; norms
1e-13 relative (fixed but different summation order); Newton / time-stepping: equal outer and inner
iteration counts, iterates to 1e-10 (the solve's own tolerance is 6e-6 absolute).
Shapes include the x-wrap corner cases of the kernels: the last column held by lane 0 of a wave
(nx = 130 with 2-wide lanes, nx = 129 with 1-wide), a 2-tile row (nx = 514) and the 3-point minimum.
"""
import numpy as np
import pytest

import _nkpath  # noqa: F401
import ariadne_hip as ah
from oracle import oracle as oc

pytestmark = pytest.mark.gpu

SCHEMES = [("euler", 0.5), ("midpoint", 0.5), ("midpoint", 0.3), ("trapezoid", 0.5)]
GNAME = {"euler": ah.G_Euler_, "midpoint": ah.G_Midpoint_, "trapezoid": ah.G_Trapezoid_}
BCS = {oc.BC_ZERO: ah.bc_zero_, oc.BC_PERIODIC: ah.bc_periodic_}
SHAPES2 = [(40, 40), (130, 67), (129, 9), (514, 5), (3, 3), (64, 33)]
SHAPES3 = [(12, 12, 12), (33, 17, 9), (130, 5, 4), (3, 3, 3), (65, 7, 5)]


@pytest.fixture(scope="module")
def ctx():
    c = ah.Context(0)
    ah.set_default_context(c)
    yield c
    c.sync()


def dev(a):
    return ah.DeviceArray.from_numpy(a)


def device_residual(P):
    scheme = {oc.HEAT2D_EULER: "euler", oc.HEAT3D_EULER: "euler", oc.HEAT2D_MIDPOINT: "midpoint",
              oc.HEAT3D_MIDPOINT: "midpoint", oc.HEAT2D_TRAPEZOID: "trapezoid", oc.HEAT3D_TRAPEZOID: "trapezoid"}[P.kind]
    G = GNAME[scheme]
    if scheme == "midpoint":
        G = G(alpha=P.alpha)
    F = G.bind(ah.diffusion_ if P.dim == 2 else ah.diffusion3d_)
    un = dev(P.un)
    fp = (P.a, P.hx, P.hy, BCS[P.bc]) if P.dim == 2 else (P.a, P.hx, P.hy, P.hz, BCS[P.bc])
    return F, (un, P.dt, None, fp, 0.0)


def cases():
    rng = np.random.default_rng(5)
    out = []
    for scheme, alpha in SCHEMES:
        for bc in (oc.BC_ZERO, oc.BC_PERIODIC):
            for shape in SHAPES2 + SHAPES3:
                un = rng.standard_normal(shape[::-1])
                mk = oc.heat2d_euler if len(shape) == 2 else oc.heat3d_euler
                P = mk(*shape, un=un, scheme=scheme, bc=bc, alpha=alpha)
                out.append(pytest.param(P, un + 0.01 * rng.standard_normal(un.shape),
                                        id=f"{scheme}{alpha if scheme == 'midpoint' else ''}-bc{bc}-{'x'.join(map(str, shape))}"))
    return out


CASES = cases()


@pytest.mark.parametrize("P,u", CASES)
def test_scheme_kernels_bitwise(ctx, P, u):
    F, p = device_residual(P)
    rng = np.random.default_rng(P.nx * 7 + P.ny)
    v = rng.standard_normal(u.shape)
    ud, vd = dev(u), dev(v)
    res, out = ud.zero(), ud.zero()
    F(res, ud, p)
    F0 = oc.residual(P, u)
    assert np.array_equal(res.to_numpy(), F0), np.max(np.abs(res.to_numpy() - F0))
    nrm = F.residual_norm(res, ud, p)
    assert abs(nrm - oc.norm(F0)) <= 1e-13 * nrm
    ah.mul_(out, ah.JacobianOperator(F, res, ud, p, jv="exact"), vd)
    assert np.array_equal(out.to_numpy(), oc.jv_exact(P, u, v))
    eps = oc.fd_eps(oc.norm(u), oc.norm(v))
    ah.mul_(out, ah.JacobianOperator(F, res, ud, p, jv="fd"), vd, eps=eps)
    assert np.array_equal(out.to_numpy(), oc.jv_fd(P, u, v, F0, eps))
    # diag(J): the exact tangent's arithmetic on unit vectors (a few probes)
    d = ah.jacobian_diag(ah.JacobianOperator(F, res, ud, p)).to_numpy().reshape(-1)
    for i in rng.integers(0, P.n, 4):
        e = np.zeros(P.n)
        e[i] = 1.0
        assert d[i] == oc.jv_exact(P, u, e.reshape(u.shape)).reshape(-1)[i]


@pytest.mark.parametrize("scheme,alpha", SCHEMES)
@pytest.mark.parametrize("bc", [oc.BC_ZERO, oc.BC_PERIODIC])
@pytest.mark.parametrize("jv", ["exact", "fd"])
def test_scheme_newton_matches_oracle(ctx, scheme, alpha, bc, jv):
    """One implicit step (newton_krylov!, tol_abs = 6e-6 as implicit.jl:67-70) from a noisy state:
    equal Newton / Krylov counts and the same iterate."""
    N = 48
    rng = np.random.default_rng(2)
    un = np.sin(np.pi * np.arange(1, N + 1) / (N + 1))[:, None] * np.ones(N)[None, :] + 0.1 * rng.uniform(-1, 1, (N, N))
    P = oc.heat2d_euler(N, un=un, scheme=scheme, bc=bc, alpha=alpha)
    F, p = device_residual(P)
    u, r = ah.newton_krylov_(F, dev(un), p, tol_abs=6e-6, jv=jv)
    uo, so = oc.newton_krylov(P, un, tol_abs=6e-6, jv=jv)
    assert r.solved and so["solved"]
    assert (r.stats.outer_iterations, r.stats.inner_iterations) == (so["outer_iterations"], so["inner_iterations"])
    assert np.max(np.abs(u.to_numpy() - uo)) <= 1e-10
    oc.set_devred(True)  # in the device's reduction order: bit for bit
    try:
        ud, _ = oc.newton_krylov(P, un, tol_abs=6e-6, jv=jv)
    finally:
        oc.set_devred(False)
    np.testing.assert_array_equal(u.to_numpy(), ud)


@pytest.mark.parametrize("G,scheme", [(ah.G_Midpoint_, "midpoint"), (ah.G_Trapezoid_, "trapezoid"), (ah.G_Euler_, "euler")])
def test_solve_timestepping_periodic(ctx, G, scheme):
    """implicit.jl `solve` with each scheme and bc_periodic! (the heat_2D.jl:150-154 configuration):
    per-step Newton/Krylov counts equal the oracle's, final state to 1e-10."""
    N = 40
    rng = np.random.default_rng(3)
    P = oc.heat2d_euler(N, scheme=scheme, bc=oc.BC_PERIODIC)
    u0 = oc.sin_ic(P) + 0.1 * rng.uniform(-1, 1, (N, N))
    ts = [i * P.dt for i in range(4)]
    un = dev(u0)
    results = []
    ah.solve(G, ah.diffusion_, un, (P.a, P.hx, P.hy, ah.bc_periodic_), P.dt, ts, stats_out=results,
             krylov_kwargs={"reorthogonalization": True})
    cur = u0.copy()
    for r in results:
        Q = oc.heat2d_euler(N, un=cur, scheme=scheme, bc=oc.BC_PERIODIC)
        cur, so = oc.newton_krylov(Q, cur, tol_abs=6e-6, reorthogonalization=True)
        assert r.solved and so["solved"]
        assert (r.stats.outer_iterations, r.stats.inner_iterations) == (so["outer_iterations"], so["inner_iterations"])
    assert np.max(np.abs(un.to_numpy() - cur)) <= 1e-10
    cur = u0.copy()  # the whole time loop in the device's reduction order: bit for bit
    oc.set_devred(True)
    try:
        for _ in results:
            cur, _ = oc.newton_krylov(oc.heat2d_euler(N, un=cur, scheme=scheme, bc=oc.BC_PERIODIC), cur, tol_abs=6e-6,
                                      reorthogonalization=True)
    finally:
        oc.set_devred(False)
    np.testing.assert_array_equal(un.to_numpy(), cur)


def test_trapezoid_periodic_eigen_decay_3d(ctx):
    """Exact Crank-Nicolson amplification of the periodic cos mode, 3D, one Krylov iteration."""
    N = 16
    c = np.cos(2 * np.pi * np.arange(N) / N)
    u0 = np.ascontiguousarray(c[:, None, None] * c[None, :, None] * c[None, None, :])
    P = oc.heat3d_euler(N, scheme="trapezoid", bc=oc.BC_PERIODIC, un=u0)
    F, p = device_residual(P)
    u, r = ah.newton_krylov_(F, dev(u0), p, tol_abs=6e-6)
    mu = -P.a * 12.0 / (P.hx * P.hx) * np.sin(np.pi / N) ** 2
    g = (1 + 0.5 * P.dt * mu) / (1 - 0.5 * P.dt * mu)
    assert r.solved and r.stats.inner_iterations == 1
    assert np.max(np.abs(u.to_numpy() - g * u0)) < 1e-10


# ----------------------------------------------------------------------------- BASELINE sizes
@pytest.mark.parametrize("dim,scheme,bc", [(2, "euler", oc.BC_ZERO), (2, "trapezoid", oc.BC_PERIODIC),
                                           (3, "euler", oc.BC_ZERO), (3, "midpoint", oc.BC_ZERO)],
                         ids=["heat2d-8192-euler", "heat2d-8192-trapezoid-periodic", "heat3d-512-euler",
                              "heat3d-512-midpoint"])
def test_heat_config_size_bitwise(ctx, dim, scheme, bc):
    """Configs 3 / 5 sizes (8192², 512³ = one GPU's bench slab): the residual and the fused FD Jv
    (the bench's kernels) on the whole grid, bit-identical to the oracle; exact-JVP linearity."""
    n = 8192 if dim == 2 else 512
    rng = np.random.default_rng(21)
    shape = (n,) * dim
    un = rng.standard_normal(shape)
    mk = oc.heat2d_euler if dim == 2 else oc.heat3d_euler
    P = mk(n, un=un, scheme=scheme, bc=bc)
    u = un + 0.01 * rng.standard_normal(shape)
    F, p = device_residual(P)
    ud = dev(u)
    res = ud.zero()
    F(res, ud, p)
    F0 = oc.residual(P, u)
    assert np.array_equal(res.to_numpy(), F0)
    del un
    v = rng.standard_normal(shape)
    vd, out = dev(v), ud.zero()
    eps = oc.fd_eps(oc.norm(u), oc.norm(v))
    ah.mul_(out, ah.JacobianOperator(F, res, ud, p, jv="fd"), vd, eps=eps)
    assert np.array_equal(out.to_numpy(), oc.jv_fd(P, u, v, F0, eps))
    J = ah.JacobianOperator(F, res, ud, p, jv="exact")
    ah.mul_(out, J, vd)
    out2 = ud.zero()
    ah.kscal_(len(vd), 2.0, vd)
    ah.mul_(out2, J, vd)
    assert np.array_equal(out2.to_numpy(), 2.0 * out.to_numpy())


@pytest.mark.parametrize("shape,scheme", [((10, 15), "midpoint"), ((7, 6), "trapezoid"), ((5, 10, 5), "euler"),
                                          ((4, 3, 5), "trapezoid")],
                         ids=["2d-colour", "2d-dense", "3d-colour", "3d-dense"])
def test_collect_periodic_matches_unit_probing(ctx, shape, scheme):
    """collect(J) with bc_periodic!: the wrap entries are present; the stencil colouring is used when
    the extents keep it distance-2 across the wrap (multiples of 2 dim + 1), unit probing otherwise;
    either way bit-identical to the oracle's exact tangent on unit vectors."""
    rng = np.random.default_rng(8)
    un = rng.standard_normal(shape[::-1])
    mk = oc.heat2d_euler if len(shape) == 2 else oc.heat3d_euler
    P = mk(*shape, un=un, scheme=scheme, bc=oc.BC_PERIODIC)
    F, p = device_residual(P)
    u = dev(un + 0.01 * rng.standard_normal(un.shape))
    J = ah.JacobianOperator(F, u.zero(), u, p)
    A = ah.collect(J).toarray()
    n = P.n
    ref = np.stack([oc.jv_exact(P, u.to_numpy(), np.eye(n)[c].reshape(un.shape)).reshape(-1) for c in range(n)], axis=1)
    np.testing.assert_array_equal(A, ref)
    np.testing.assert_array_equal(ah.collect(J.T).toarray(), ref.T)
