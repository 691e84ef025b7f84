"""How close the device Bratu path is to the oracle now that both use nk_exp (csrc/nk_exp.h): prints the
number of differing elements of the residual / exact JVP / FD operator at several sizes, and the
largest relative differences of GMRES histories and iterates (the quantities tests/test_hip.py bounds).

    python tools/bratu_parity_probe.py          (GPU box; results on stdout)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _nkpath  # noqa: E402,F401
import ariadne_hip as ah  # noqa: E402
from oracle import oracle as oc  # noqa: E402


def dev(a):
    return ah.DeviceArray.from_numpy(a)


def kernels(n, m=None):
    P = oc.bratu2d(n, m)
    rng = np.random.default_rng(1)
    u = oc.sin_ic(P) + 0.05 * rng.standard_normal(P.shape)
    v = rng.standard_normal(P.shape)
    p = (P.hx, P.hy, P.lam)
    ud, vd = dev(u), dev(v)
    res, out = ud.zero(), ud.zero()
    ah.bratu2d_(res, ud, p)
    F0 = res.to_numpy()
    r_res = np.sum(F0 != oc.residual(P, u))
    ah.mul_(out, ah.JacobianOperator(ah.bratu2d_, res, ud, p, jv="exact"), vd)
    r_jv = np.sum(out.to_numpy() != oc.jv_exact(P, u, v))
    eps = oc.fd_eps(oc.norm(u), oc.norm(v))
    ah.mul_(out, ah.JacobianOperator(ah.bratu2d_, res, ud, p, jv="fd"), vd, eps=eps)
    r_fd = np.sum(out.to_numpy() != oc.jv_fd(P, u, v, F0, eps))
    print(f"{n}x{m or n}: residual differs at {r_res}, exact JVP at {r_jv}, FD at {r_fd} of {P.n} points", flush=True)


def gmres(restart, memory, reorth, jv, n=24):
    P = oc.bratu2d(n)
    u = oc.sin_ic(P)
    b = oc.residual(P, u)
    kw = dict(restart=restart, reorthogonalization=reorth, atol=1e-12, rtol=1e-9, itmax=150)
    ud, bd = dev(u), dev(b)
    res = ud.zero()
    ah.bratu2d_(res, ud, (P.hx, P.hy, P.lam))
    ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=memory))
    J = ah.JacobianOperator(ah.bratu2d_, res, ud, (P.hx, P.hy, P.lam), jv=jv)
    ah.krylov_solve_(ws, J, bd, history=True, **kw)
    x, st = ws.x.to_numpy(), ws.stats
    xo, so, ho = oc.krylov_solve(P, u, b, jv=jv, F0=res.to_numpy(), memory=memory, **kw)
    h = np.array(st.residuals)
    k = ho > 1e-6 * ho[0]
    rel = np.max(np.abs(h[k] - ho[k]) / ho[k])
    print(f"gmres restart={restart} mem={memory} reorth={reorth} jv={jv}: niter {st.niter}/{so['niter']} "
          f"hist rel {rel:.2e} first-cycle {np.max(np.abs(h[:memory + 1] - ho[:memory + 1]) / ho[:memory + 1]):.2e} "
          f"x rel {np.max(np.abs(x - xo)) / np.max(np.abs(xo)):.2e}", flush=True)


def newton(n=64):
    P = oc.bratu2d(n)
    u0 = oc.sin_ic(P)
    for jv in ("exact", "fd"):
        u, r = ah.newton_krylov_(ah.bratu2d_, dev(u0), (P.hx, P.hy, P.lam), memory=30, tol_rel=1e-10,
                                 krylov_kwargs=dict(restart=True), jv=jv)
        uo, so = oc.newton_krylov(P, u0, memory=30, restart=True, tol_rel=1e-10, jv=jv)
        uu = u.to_numpy()
        print(f"newton {n}^2 jv={jv}: outer {r.stats.outer_iterations}/{so['outer_iterations']} inner "
              f"{r.stats.inner_iterations}/{so['inner_iterations']} u rel {np.max(np.abs(uu - uo)) / np.max(np.abs(uo)):.2e} "
              f"||F|| dev {r.stats.n_res:.6e} oracle-on-dev-iterate {oc.norm(oc.residual(P, uu)):.6e}", flush=True)


def main():
    ctx = ah.Context(0)
    ah.set_default_context(ctx)
    for n, m in ((64, None), (63, 37), (1000, 5), (4096, None)):
        kernels(n, m)
    for cfg in ((False, 20, False, "exact"), (True, 10, False, "exact"), (True, 8, True, "exact"), (True, 10, False, "fd"),
                (False, 20, False, "fd"), (True, 8, True, "fd")):
        gmres(*cfg)
    newton()


if __name__ == "__main__":
    main()
