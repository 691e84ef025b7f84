"""GPU-vs-oracle divergence of FD-GMRES (diagnostic; prints the numbers the FD tolerances in
tests/test_hip.py are set from).  Not part of the product."""
import sys

import numpy as np

sys.path.insert(0, '.')
import _nkpath  # noqa: F401,E402
import ariadne_hip as ah  # noqa: E402
from oracle import oracle as oc  # noqa: E402

ctx = ah.Context(0)
ah.set_default_context(ctx)


def run(P, u, F, p, restart, mem, un=None):
    b = oc.residual(P, u)
    ud = ah.DeviceArray.from_numpy(u)
    res = ud.zero()
    F(res, ud, p)
    ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=mem))
    J = ah.JacobianOperator(F, res, ud, p, jv="fd")
    kw = dict(restart=restart, atol=1e-12, rtol=1e-9, itmax=150)
    ah.krylov_solve_(ws, J, ah.DeviceArray.from_numpy(b), history=True, **kw)
    x, h, F0 = ws.x.to_numpy(), np.array(ws.stats.residuals), res.to_numpy()
    ws.free()
    xo, so, ho = oc.krylov_solve(P, u, b, jv="fd", F0=F0, memory=mem, **kw)
    oc.set_chunk(7)
    xc, sc, hc = oc.krylov_solve(P, u, b, jv="fd", F0=F0, memory=mem, **kw)
    oc.set_chunk(8192)
    m = min(len(h), len(ho), len(hc))
    out = [f"niter {len(h) - 1}/{so['niter']}"]
    for thr in (1e-2, 1e-4, 1e-6):
        k = ho[:m] > thr * ho[0]
        out.append(f"hist>{thr:g}: gpu {np.max(np.abs(h[:m] - ho[:m])[k] / ho[:m][k]):.1e} "
                   f"cpu-cpu {np.max(np.abs(hc[:m] - ho[:m])[k] / ho[:m][k]):.1e}")
    out.append(f"x: gpu {np.max(np.abs(x - xo)) / np.max(np.abs(xo)):.1e} cpu-cpu {np.max(np.abs(xc - xo)) / np.max(np.abs(xo)):.1e}")
    return "  ".join(out)


for n, restart, mem in ((24, True, 10), (24, False, 20), (40, True, 10)):
    P = oc.bratu2d(n)
    print("bratu2d", n, restart, mem, run(P, oc.sin_ic(P), ah.bratu2d_, (P.hx, P.hy, P.lam), restart, mem))
for n, restart, mem in ((24, True, 10), (24, False, 20)):
    P = oc.bratu2d(n)
    u0 = oc.sin_ic(P) + 0.1 * np.random.default_rng(1).standard_normal(P.shape)
    un = u0.copy()
    P = oc.heat2d_euler(n, un=un)
    und = ah.DeviceArray.from_numpy(un)
    p = (und, P.dt, None, (P.a, P.hx, P.hy, ah.bc_zero_), 0.0)
    F = ah.G_Euler_.bind(ah.diffusion_)
    print("heat2d", n, restart, mem, run(P, u0 + 0.01, F, p, restart, mem))
