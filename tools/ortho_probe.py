"""Full-size Arnoldi-cycle properties (diagnostic; prints the numbers the tolerances of
tests/test_hip_resident.py::test_full_size_cycle_properties are set from).  Not part of the product."""
import sys

import numpy as np

sys.path.insert(0, '.')
import _nkpath  # noqa: F401,E402
import ariadne_hip as ah  # noqa: E402

ctx = ah.Context(0)
ah.set_default_context(ctx)
for n, jv, reorth in ((4096, "exact", False), (4096, "fd", False), (4096, "exact", True)):
    h = 1.0 / (n + 1)
    xs = np.arange(1, n + 1) * h
    u0 = np.sin(np.pi * xs)[:, None] * np.sin(np.pi * xs)[None, :]
    u = ah.DeviceArray.from_numpy(u0)
    res = u.zero()
    p = (h, h, 3.51382)
    ah.bratu2d_(res, u, p)
    J = ah.JacobianOperator(ah.bratu2d_, res, u, p, jv=jv)
    ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=30))
    ctx.prof_reset()
    ctx.prof_enable(1)
    ah.krylov_solve_(ws, J, res, restart=True, itmax=60, atol=0.0, rtol=0.0, history=True, reorthogonalization=reorth)
    prof = ctx.prof_read()
    ctx.prof_enable(0)
    hist = ws.stats.residuals
    V = [ws.basis(i) for i in range(30)]
    N = len(u)
    G = np.array([[ah.kdot(N, V[i], V[j]) for j in range(30)] for i in range(30)])
    orth = np.max(np.abs(G - np.eye(30)))
    Jx = u.zero()
    ah.mul_(Jx, J, ws.x)
    r = res.copy()
    ah.kaxpy_(N, -1.0, Jx, r)
    true = ah.knorm(N, r)
    print(f"{n}^2 jv={jv} reorth={reorth} sweeps={prof.get('mgs_sweep', {}).get('launches')} niter={ws.stats.niter} "
          f"orth={orth:.2e} est={hist[-1]:.12e} true={true:.12e} rel={abs(true - hist[-1]) / hist[-1]:.2e} "
          f"r0={hist[0]:.6e}")
    ws.free()
