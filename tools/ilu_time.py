"""Time the ILU(0) factor and one z = (L U)^-1 v at 2D Bratu n^2 (pipelined vs level sweeps: run
twice, with NK_ILU_PIPE=0 for the level form).  Usage: python tools/ilu_time.py [n]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import _nkpath  # noqa: F401,E402
import ariadne_hip as ah  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
ctx = ah.Context(0)
ah.set_default_context(ctx)
h = 1.0 / (n + 1)
x = np.sin(np.pi * np.arange(1, n + 1) * h)
u = ah.DeviceArray.from_numpy(np.outer(x, x))
J = ah.JacobianOperator(ah.bratu2d_, u.zero(), u, (h, h, 3.51382))
v = ah.DeviceArray.from_numpy(np.random.default_rng(0).standard_normal((n, n)))
N = ah.ilu0(J)
ctx.sync()
ctx.prof_reset()
ctx.prof_enable(1)
for _ in range(3):
    N = ah.ilu0(J)
    z = N.apply(J, v)
ctx.sync()
prof = ctx.prof_read()
ctx.prof_enable(0)
print(f"ILU(0) at {n}^2 (NK_ILU_PIPE={os.environ.get('NK_ILU_PIPE', '1')}):")
for k, e in sorted(prof.items()):
    if k.startswith("ilu0"):
        print(f"  {k:20s} {e['ms'] / max(1, e['timed']):9.3f} ms per launch ({e['timed']} timed)")
