"""GPU tests of nk_newton_krylov (the Newton loop of src/Ariadne.jl:288-372 inside libnkhip.so, the
entry point for C / C++ callers).  It issues exactly the library calls the Python host mirror issues,
so every result must be BIT-IDENTICAL to `newton_krylov_`; against the CPU oracle: equal outer/inner
counts, and the root bit for bit in the oracle's device-order mode."""
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


CASES = [
    dict(jv="exact", forcing=ah.EisenstatWalker(), algo="gmres", memory=20, krylov_kwargs={}),
    dict(jv="fd", forcing=ah.EisenstatWalker(), algo="gmres", memory=10, krylov_kwargs=dict(restart=True)),
    dict(jv="exact", forcing=ah.Fixed(0.05), algo="gmres", memory=20, krylov_kwargs=dict(reorthogonalization=True)),
    dict(jv="fd", forcing=None, algo="gmres", memory=30, krylov_kwargs=dict(restart=True, itmax=60)),
    dict(jv="exact", forcing=ah.EisenstatWalker(), algo="gmres", memory=20, krylov_kwargs=dict(rtol=1e-3)),
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_native_newton_bit_identical_to_host_loop(ctx, case):
    kw = CASES[case]
    P = oc.bratu2d(96, 72)
    u0 = oc.sin_ic(P)
    p = (P.hx, P.hy, P.lam)
    ua, ra = ah.newton_krylov_(ah.bratu2d_, ah.DeviceArray.from_numpy(u0), p, **kw)
    ub, rb = ah.newton_krylov_native(ah.bratu2d_, ah.DeviceArray.from_numpy(u0), p, **kw)
    assert ra.solved == rb.solved
    assert ra.stats == rb.stats
    assert ra.n_matvec == rb.n_matvec
    np.testing.assert_array_equal(ua.to_numpy(), ub.to_numpy())


def test_native_newton_cg_bratu1d_matches_oracle(ctx):
    """Config 1 (examples/bratu.jl:59-63): algo = :cg on 1D Bratu N = 1000 -- against the oracle in the
    device's reduction order (test_hip_devred.py): equal counts and the root bit for bit."""
    P = oc.bratu1d(1000)
    u0 = oc.sin_ic(P)
    oc.set_devred(True)
    try:
        ref, st = oc.newton_krylov(P, u0, algo="cg")
    finally:
        oc.set_devred(False)
    u, r = ah.newton_krylov_native(ah.bratu_, ah.DeviceArray.from_numpy(u0), (P.hx, P.lam), algo="cg")
    assert r.solved and st["solved"]
    assert (r.stats.outer_iterations, r.stats.inner_iterations) == (st["outer_iterations"], st["inner_iterations"])
    np.testing.assert_array_equal(u.to_numpy(), ref)


def test_native_newton_heat_step_matches_oracle(ctx):
    rng = np.random.default_rng(1)
    un = rng.standard_normal((48, 64))
    P = oc.heat2d_euler(64, 48, un=un)
    u0 = un.copy()
    ref, st = oc.newton_krylov(P, u0, tol_abs=6e-6, memory=20)
    p = (ah.DeviceArray.from_numpy(un), P.dt, None, (P.a, P.hx, P.hy, ah.bc_zero_), 0.0)
    u, r = ah.newton_krylov_native(ah.heat2d_euler_, ah.DeviceArray.from_numpy(u0), p, tol_abs=6e-6, memory=20)
    assert r.solved and st["solved"]
    assert (r.stats.outer_iterations, r.stats.inner_iterations) == (st["outer_iterations"], st["inner_iterations"])
    np.testing.assert_allclose(u.to_numpy(), ref, rtol=0, atol=1e-10 * np.abs(ref).max())
    oc.set_devred(True)  # and in the device's reduction order: bit for bit
    try:
        ref_dev, _ = oc.newton_krylov(P, u0, tol_abs=6e-6, memory=20)
    finally:
        oc.set_devred(False)
    np.testing.assert_array_equal(u.to_numpy(), ref_dev)


def test_native_newton_user_residual(ctx):
    """The native loop drives a user residual too (NK_USER2D): same result as the built-in kernel."""
    import torch

    def heat(res, u, p):
        un, dt, _du, (a, hx, hy, _bc), _t = p
        Q = torch.nn.functional.pad(u.torch(ghosts=True), (1, 1))
        c = Q[1:-1, 1:-1]
        h2x = torch.tensor(hx * hx, dtype=Q.dtype, device=Q.device)
        h2y = torch.tensor(hy * hy, dtype=Q.dtype, device=Q.device)
        lsum = ((Q[1:-1, 2:] - 2.0 * c) + Q[1:-1, :-2]) / h2x + ((Q[2:, 1:-1] - 2.0 * c) + Q[:-2, 1:-1]) / h2y
        res.torch().copy_((un.torch() + dt * (a * lsum)) - c)

    rng = np.random.default_rng(2)
    un = rng.standard_normal((40, 56))
    P = oc.heat2d_euler(56, 40, un=un)
    p = (ah.DeviceArray.from_numpy(un), P.dt, None, (P.a, P.hx, P.hy, ah.bc_zero_), 0.0)
    ua, ra = ah.newton_krylov_native(ah.UserResidual(heat), ah.DeviceArray.from_numpy(un), p, tol_abs=6e-6, jv="fd")
    ub, rb = ah.newton_krylov_native(ah.heat2d_euler_, ah.DeviceArray.from_numpy(un), p, tol_abs=6e-6, jv="fd")
    assert ra.stats.outer_iterations == rb.stats.outer_iterations and ra.solved and rb.solved
    # the reductions are summed in a different (fixed) order on the two paths; a solve to tol_abs = 6e-6
    # leaves that visible at ~1e-11
    np.testing.assert_allclose(ua.to_numpy(), ub.to_numpy(), rtol=0, atol=1e-9 * np.abs(un).max())
    # each path bit for bit against the oracle in its own device order: the user residual's reductions are
    # k_user_epi's scalar chunks (oracle.set_devred(user=True)), the built-in stencil's its tiles
    for u_dev, r_dev, user in ((ua, ra, True), (ub, rb, False)):
        oc.set_devred(True, user=user)
        try:
            uo, so = oc.newton_krylov(P, un, tol_abs=6e-6, jv="fd")
        finally:
            oc.set_devred(False)
        assert (r_dev.stats.outer_iterations, r_dev.stats.inner_iterations) == (so["outer_iterations"], so["inner_iterations"])
        np.testing.assert_array_equal(u_dev.to_numpy(), uo)
