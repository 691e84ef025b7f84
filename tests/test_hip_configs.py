"""GPU parity at the per-rank sizes of the multi-GPU configurations, on one GPU.

BASELINE.json configs[3] (2D Bratu 16384^2 over 8 GPUs: a 16384 x 2048 slab per rank) and
configs[4] (3D heat 512^3 over 8 GPUs: a 512^2 x 64 z-slab per rank) run on the 8-GPU node only;
these tests run exactly one rank's slab of each on the test box's one GPU, with its ghost planes
filled by hand from the neighbouring rows / planes of the global field (what the halo exchange
delivers), against the oracle on the slab plus its two ghost planes:

* config-4 slab (rank 3 of 8): residual, exact and FD JVP bit for bit (the device and the oracle share
  the correctly rounded exp, csrc/nk_exp.h); then the first 12 FD-GMRES(30) Arnoldi steps of the slab
  problem (global h, zero ghosts: the Dirichlet slab) against the oracle -- half of q resident in the
  sweep -- to the reductions' summation order;
* the whole 16384^2 problem on one GPU (268 M points, 2.1 GB per vector, byte offsets past 2^31):
  residual and exact JVP bit for bit;
* config-5 slab (rank 3 of 8), every implicit scheme: residual, exact and FD JVP bit for bit, and
  one implicit-Euler time step of the Dirichlet slab with equal Newton / Krylov counts.
"""
import ctypes as C

import numpy as np
import pytest

import _nkpath  # noqa: F401
import ariadne_hip as ah
from ariadne_hip import _lib
from oracle import oracle as oc

pytestmark = pytest.mark.gpu
ULP = np.finfo(np.float64).eps
LAM = 3.51382


@pytest.fixture(scope="module")
def ctx():
    c = ah.Context(0)
    ah.set_default_context(c)
    yield c
    c.sync()


def set_ghosts(d, ext):
    """Write ext[0] / ext[-1] (planes along the slowest axis) into d's lower / upper ghost plane."""
    plane = int(np.prod(d.grid.np_shape[1:]))
    lo = np.ascontiguousarray(ext[0], dtype=np.float64)
    hi = np.ascontiguousarray(ext[-1], dtype=np.float64)
    lib = _lib.load()
    d.ctx.check(lib.nk_memcpy_h2d(d.ctx.handle, d.ptr - 8 * plane, lo.ctypes.data, plane), "ghost lo")
    d.ctx.check(lib.nk_memcpy_h2d(d.ctx.handle, d.ptr + 8 * d.n, hi.ctypes.data, plane), "ghost hi")


def with_ghosts(ext, grid, ctx):
    d = ah.DeviceArray.from_numpy(np.ascontiguousarray(ext[1:-1]), grid, ctx)
    set_ghosts(d, ext)
    return d


# ----------------------------------------------------------------------------- config 4
N4, WORLD, RANK = 16384, 8, 3


def config4_slab():
    rows = N4 // WORLD
    y0 = RANK * rows
    h = 1.0 / (N4 + 1)
    xs = np.arange(1, N4 + 1) * h
    ys = np.arange(y0, y0 + rows + 2) * h  # global rows y0-1 .. y0+rows (ghosts included)
    u_ext = np.sin(np.pi * ys)[:, None] * np.sin(np.pi * xs)[None, :]
    grid = ah.Grid((N4, rows), (N4, N4), y0)
    return grid, h, u_ext


def test_config4_slab_kernels_with_ghosts(ctx):
    grid, h, u_ext = config4_slab()
    rows = grid.shape_xyz[1]
    v_ext = np.random.default_rng(4).standard_normal(u_ext.shape)
    Pext = oc.Problem(oc.BRATU2D, N4, rows + 2, hx=h, hy=h, lam=LAM)
    p = (h, h, LAM)
    u, v = with_ghosts(u_ext, grid, ctx), with_ghosts(v_ext, grid, ctx)
    res = u.zero()
    ah.bratu2d_(res, u, p)
    F = res.to_numpy()
    Fo = oc.residual(Pext, u_ext)[1:-1]
    np.testing.assert_array_equal(F, Fo)  # ghost rows taken from the "neighbours"
    out = u.zero()
    ah.mul_(out, ah.JacobianOperator(ah.bratu2d_, res, u, p, jv="exact"), v)
    np.testing.assert_array_equal(out.to_numpy(), oc.jv_exact(Pext, u_ext, v_ext)[1:-1])
    eps = 1e-7
    ah.mul_(out, ah.JacobianOperator(ah.bratu2d_, res, u, p, jv="fd"), v, eps=eps)
    F0ext = np.concatenate([np.zeros((1, N4)), F, np.zeros((1, N4))])  # the device's F(u), as the operator uses it
    np.testing.assert_array_equal(out.to_numpy(), oc.jv_fd(Pext, u_ext, v_ext, F0=F0ext, eps=eps)[1:-1])


def test_config4_slab_gmres_first_steps(ctx):
    """The rank's Dirichlet slab problem (global h, zero ghosts): 12 FD-GMRES(30) steps vs the oracle."""
    grid, h, u_ext = config4_slab()
    rows = grid.shape_xyz[1]
    # a state that vanishes on the slab's zero ghosts (sin(pi x) sin(pi j / (rows + 1))): the global
    # profile would jump to 0 there (F ~ u / h^2 ~ 2.5e8 at the edge rows)
    ys = np.sin(np.pi * np.arange(1, rows + 1) / (rows + 1))
    ui = np.ascontiguousarray(ys[:, None] * np.sin(np.pi * np.arange(1, N4 + 1) * h)[None, :])
    P = oc.Problem(oc.BRATU2D, N4, rows, hx=h, hy=h, lam=LAM)
    p = (h, h, LAM)
    u = ah.DeviceArray.from_numpy(ui, grid, ctx)
    res = u.zero()
    ah.bratu2d_(res, u, p)
    F0d = res.to_numpy()
    ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=30))
    ctx.prof_reset()
    ctx.prof_enable(1 << 20)
    kw = dict(restart=True, atol=0.0, rtol=0.0, itmax=12)
    ah.krylov_solve_(ws, ah.JacobianOperator(ah.bratu2d_, res, u, p, jv="fd"), res, history=True, **kw)
    sweep = ctx.prof_read().get("mgs_sweep", {})
    sweeps = sweep.get("launches", 0)
    ctx.prof_enable(0)
    assert sweeps > 0, "the (half-resident) MGS sweep did not run"
    # the profile names the instantiation that ran, as rocprofv3 does: half of q streams, non-temporally
    assert sweep["kernel"] == "nk::k_mgs_res<89, 4, true, false, false, 0, true, 4>", sweep["kernel"]
    x = ws.x.to_numpy()
    xo, sto, ho = oc.krylov_solve(P, ui, F0d, jv="fd", F0=F0d, memory=30, **kw)
    assert ws.stats.niter == sto["niter"] == 12
    # the operator is bit-identical: only the summation order of the reductions differs.  The residual
    # histories follow it to 1e-11; x, to the FD operator's own noise: a one-ulp change in a basis vector
    # moves F(u + eps v)'s roundings, |F| / |Jv| ~ 1e3 here, so Jv moves by ~1e-16 |F| / eps ~ 1e-9 |Jv|,
    # and x, made of the V_k, follows (measured 9.9e-9 relative on the GPU, r04)
    assert np.allclose(np.array(ws.stats.residuals), ho, rtol=1e-11)
    assert np.max(np.abs(x - xo)) <= 5e-8 * np.max(np.abs(xo))
    oc.set_devred(True, cus=ctx.path_info()["resident_blocks"] or 256)  # the half-resident sweep's own order
    try:
        xr, _, hr = oc.krylov_solve(P, ui, F0d, jv="fd", F0=F0d, memory=30, **kw)
    finally:
        oc.set_devred(False)
    np.testing.assert_array_equal(np.array(ws.stats.residuals), hr)
    np.testing.assert_array_equal(x, xr)
    ws.free()


def test_bratu2d_16384_on_one_gpu(ctx):
    """The whole config-4 grid on one GPU: 268 M points (byte offsets beyond 2^31)."""
    P = oc.bratu2d(N4)
    u0 = oc.sin_ic(P)
    p = (P.hx, P.hy, P.lam)
    u = ah.DeviceArray.from_numpy(u0, None, ctx)
    res = u.zero()
    ah.bratu2d_(res, u, p)
    np.testing.assert_array_equal(res.to_numpy(), oc.residual(P, u0))
    v0 = np.random.default_rng(2).standard_normal(u0.shape)
    v = ah.DeviceArray.from_numpy(v0, None, ctx)
    out = res  # reuse the allocation
    ah.mul_(out, ah.JacobianOperator(ah.bratu2d_, res, u, p, jv="exact"), v)
    np.testing.assert_array_equal(out.to_numpy(), oc.jv_exact(P, u0, v0))


# ----------------------------------------------------------------------------- config 5
N5 = 512


def config5_slab(scheme):
    planes = N5 // WORLD
    z0 = RANK * planes
    rng = np.random.default_rng(5)
    h = 1.0 / (N5 + 1)
    xs = np.sin(np.pi * np.arange(1, N5 + 1) * h)
    zs = np.sin(np.pi * np.arange(z0, z0 + planes + 2) * h)
    un_ext = zs[:, None, None] * xs[None, :, None] * xs[None, None, :] + 0.1 * rng.uniform(-1, 1, (planes + 2, N5, N5))
    u_ext = un_ext + 0.01 * rng.standard_normal(un_ext.shape)
    grid = ah.Grid((N5, N5, planes), (N5, N5, N5), z0)
    dt = oc.heat_dt_3d(h, h, h, 0.01)
    Pext = oc.Problem(oc.HEAT_KINDS[scheme, 3], N5, N5, planes + 2, hx=h, hy=h, hz=h, a=0.01, dt=dt, un=un_ext,
                      alpha=0.3 if scheme == "midpoint" else 0.5)
    return grid, h, dt, un_ext, u_ext, Pext


@pytest.mark.parametrize("scheme", ["euler", "midpoint", "trapezoid"])
def test_config5_slab_kernels_bitwise(ctx, scheme):
    grid, h, dt, un_ext, u_ext, Pext = config5_slab(scheme)
    un = with_ghosts(un_ext, grid, ctx)  # G_Midpoint! / G_Trapezoid! read u_n's neighbours too
    u = with_ghosts(u_ext, grid, ctx)
    v_ext = np.random.default_rng(6).standard_normal(u_ext.shape)
    v = with_ghosts(v_ext, grid, ctx)
    G = {"euler": ah.G_Euler_, "midpoint": ah.G_Midpoint_(alpha=0.3), "trapezoid": ah.G_Trapezoid_}[scheme]
    F = G.bind(ah.diffusion3d_)
    p = (un, dt, None, (0.01, h, h, h, ah.bc_zero_), 0.0)
    res = u.zero()
    F(res, u, p)
    np.testing.assert_array_equal(res.to_numpy(), oc.residual(Pext, u_ext)[1:-1])
    out = u.zero()
    ah.mul_(out, ah.JacobianOperator(F, res, u, p, jv="exact"), v)
    np.testing.assert_array_equal(out.to_numpy(), oc.jv_exact(Pext, u_ext, v_ext)[1:-1])
    eps = 3e-8
    ah.mul_(out, ah.JacobianOperator(F, res, u, p, jv="fd"), v, eps=eps)
    F0ext = np.concatenate([np.zeros((1, N5, N5)), res.to_numpy(), np.zeros((1, N5, N5))])
    np.testing.assert_array_equal(out.to_numpy(), oc.jv_fd(Pext, u_ext, v_ext, F0=F0ext, eps=eps)[1:-1])


def test_config5_slab_time_step(ctx):
    """One implicit-Euler step (newton_krylov!, tol_abs = 6e-6, GMRES memory 20) of the rank's
    Dirichlet slab: equal Newton / Krylov counts, iterate to 1e-10."""
    grid, h, dt, un_ext, _, _ = config5_slab("euler")
    u0 = np.ascontiguousarray(un_ext[1:-1])
    un = ah.DeviceArray.from_numpy(u0, grid, ctx)
    u = un.copy()
    p = (un, dt, None, (0.01, h, h, h, ah.bc_zero_), 0.0)
    u, r = ah.newton_krylov_(ah.G_Euler_.bind(ah.diffusion3d_), u, p, tol_abs=6e-6)
    P = oc.Problem(oc.HEAT3D_EULER, N5, N5, grid.shape_xyz[2], hx=h, hy=h, hz=h, a=0.01, dt=dt, un=u0)
    uo, so = oc.newton_krylov(P, u0.copy(), tol_abs=6e-6)
    assert r.solved and so["solved"]
    assert (r.stats.outer_iterations, r.stats.inner_iterations) == (so["outer_iterations"], so["inner_iterations"])
    assert np.max(np.abs(u.to_numpy() - uo)) <= 1e-10
    oc.set_devred(True, cus=ctx.path_info()["resident_blocks"] or 256)  # the slab's own reduction trees: bitwise
    try:
        ud, _ = oc.newton_krylov(P, u0.copy(), tol_abs=6e-6)
    finally:
        oc.set_devred(False)
    np.testing.assert_array_equal(u.to_numpy(), ud)
