"""Probe (round 6): the 2D Bratu FD Jv at 4096^2 with and without its fused <V_1, Jv> (k_st2d EPI_NONE vs
EPI_DOT) -- device time per launch from the library's profile (HIP events)."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _nkpath  # noqa: F401,E402
import numpy as np  # noqa: E402
import ariadne_hip as ah  # noqa: E402
from oracle import oracle as oc  # noqa: E402

ctx = ah.Context(0)
ah.set_default_context(ctx)
P = oc.bratu2d(4096)
u = ah.DeviceArray.from_numpy(oc.sin_ic(P))
v = ah.DeviceArray.from_numpy(np.random.default_rng(1).standard_normal(P.shape))
w = ah.DeviceArray.from_numpy(np.random.default_rng(2).standard_normal(P.shape))
p = (P.hx, P.hy, P.lam)
res, out = u.zero(), u.zero()
ah.bratu2d_(res, u, p)
J = ah.JacobianOperator(ah.bratu2d_, res, u, p, jv="fd")
for it in range(3):
    ctx.prof_reset()
    ctx.prof_enable(1 << 20)
    for _ in range(50):
        ah.mul_(out, J, v, eps=1e-7)
    ctx.sync()
    a = ctx.prof_read()
    ctx.prof_reset()
    for _ in range(50):
        ah.kdot(len(out), w, out)  # (a separate dot, for scale)
    ctx.sync()
    b = ctx.prof_read()
    ctx.prof_enable(0)
    for name, d in sorted(a.items()):
        print("round", it, "mul_", name, d.get("kernel"), round(1e3 * d["ms"] / max(1, d["timed"]), 2), d["launches"], flush=True)
    for name, d in sorted(b.items()):
        print("round", it, "kdot", name, d.get("kernel"), round(1e3 * d["ms"] / max(1, d["timed"]), 2), d["launches"], flush=True)
