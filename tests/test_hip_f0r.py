"""GPU tests of the FD operator with F0 recomputed (nk_krylov_opts.f0_is_residual): in the Newton loop
F0 = res is exactly F(u) as the device residual kernel computed it, so the 2D FD stencils evaluate
F(u) again from the u rows they load anyway -- the same cooked field, Laplacian and point formula as
the residual kernel -- instead of reading F0 (8 B/pt less).  The bar is bits: whole restarted
FD-GMRES solves (Arnoldi steps with the fused V_k = q / h, the restart residual b - J x, the k = 1
and reorthogonalised steps) with and without the flag give identical histories and iterates, for
every heat scheme in 2D and 3D (k_st2d, k_st3l), zero and periodic boundaries, VEC 2 and VEC 1 (odd
nx) tiles, tiles with and without LDS y-neighbours and halo rows -- under the default policy (2D heat,
2D Bratu's Jv launches that also store V_k, 3D G_Euler!) and forced everywhere (NK_F0R=2: Bratu's
plain Jv and restart residual, whose second exp per point makes them slower, and the 3D kernels that
lose a wave per SIMD)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import _nkpath  # noqa: F401
import ariadne_hip as ah
from oracle import oracle as oc

pytestmark = pytest.mark.gpu

GNAME = {"euler": ah.G_Euler_, "midpoint": ah.G_Midpoint_, "trapezoid": ah.G_Trapezoid_}


@pytest.fixture(scope="module")
def ctx():
    c = ah.Context(0)
    ah.set_default_context(c)
    yield c
    c.sync()


def case(name, nx, ny, bc="zero", nz=0):
    rng = np.random.default_rng(nx * 7 + ny)
    if nz:  # 3D heat (k_st3l)
        un = rng.standard_normal((nz, ny, nx))
        scheme, alpha = (name.split(":") + ["0.5"])[:2]
        P = oc.heat3d_euler(nx, ny, nz, un=un, scheme=scheme, bc=oc.BC_PERIODIC if bc == "periodic" else oc.BC_ZERO,
                            alpha=float(alpha))
        G = GNAME[scheme]
        if scheme == "midpoint":
            G = G(alpha=float(alpha))
        F = G.bind(ah.diffusion3d_)
        p = (ah.DeviceArray.from_numpy(un), P.dt, None,
             (P.a, P.hx, P.hy, P.hz, ah.bc_periodic_ if bc == "periodic" else ah.bc_zero_), 0.0)
        return F, p, un + 0.01 * rng.standard_normal(un.shape)
    if name == "bratu2d":
        P = oc.bratu2d(nx, ny)
        u0 = oc.sin_ic(P) + 0.05 * rng.standard_normal(P.shape)
        return ah.bratu2d_, (P.hx, P.hy, P.lam), u0
    un = rng.standard_normal((ny, nx))
    scheme, alpha = (name.split(":") + ["0.5"])[:2]
    P = oc.heat2d_euler(nx, ny, un=un, scheme=scheme, bc=oc.BC_PERIODIC if bc == "periodic" else oc.BC_ZERO,
                        alpha=float(alpha))
    G = GNAME[scheme]
    if scheme == "midpoint":
        G = G(alpha=float(alpha))
    F = G.bind(ah.diffusion_)
    p = (ah.DeviceArray.from_numpy(un), P.dt, None,
         (P.a, P.hx, P.hy, ah.bc_periodic_ if bc == "periodic" else ah.bc_zero_), 0.0)
    return F, p, un + 0.01 * rng.standard_normal(un.shape)


def solve(F, p, u0, flag, **kw):
    u = ah.DeviceArray.from_numpy(u0)
    res = u.zero()
    F(res, u, p)
    ws = ah.krylov_workspace("gmres", ah.KrylovConstructor(res, memory=kw.pop("memory", 10)))
    J = ah.JacobianOperator(F, res, u, p, jv="fd")
    u.ctx.prof_reset()
    u.ctx.prof_enable(1)
    before = u.ctx.path_info()
    ah.krylov_solve_(ws, J, res, history=True, _f0_is_residual=flag, **kw)
    after = u.ctx.path_info()
    prof = u.ctx.prof_read()
    u.ctx.prof_enable(0)
    # the FD stencil launches by the instantiation that ran (nk_path_info launch counters)
    prof["_ran"] = {k: after[k] - before[k] for k in ("jv_fd_f0r", "jv_fd_f0_read")}
    out = ws.x.to_numpy(), list(ws.stats.residuals), ws.stats.niter, prof
    ws.free()
    return out


CASES = [("euler", 130, 67, "zero"), ("euler", 201, 37, "zero"), ("bratu2d", 200, 150, "zero"),
         ("midpoint:0.3", 130, 67, "zero"), ("trapezoid", 129, 40, "zero"), ("euler", 64, 64, "periodic"),
         ("midpoint", 96, 40, "periodic"), ("trapezoid", 65, 33, "periodic")]


CASES3 = [("euler", 40, 33, "zero", 20), ("midpoint:0.3", 33, 17, "zero", 9), ("trapezoid", 65, 7, "zero", 5),
          ("euler", 24, 24, "periodic", 24), ("trapezoid", 33, 17, "periodic", 9)]


@pytest.mark.parametrize("name,nx,ny,bc,nz", [c + (0,) for c in CASES] + CASES3)
@pytest.mark.parametrize("reorth", [False, True])
def test_f0_recomputed_is_bitwise(ctx, name, nx, ny, bc, nz, reorth):
    F, p, u0 = case(name, nx, ny, bc, nz)
    kw = dict(restart=True, memory=10, itmax=35, atol=0.0, rtol=0.0, reorthogonalization=reorth)
    x0, h0, n0, p0 = solve(F, p, u0, False, **kw)
    x1, h1, n1, p1 = solve(F, p, u0, True, **kw)
    assert n0 == n1 == 35
    assert h0 == h1
    np.testing.assert_array_equal(x0, x1)
    # the flag reached the stencils the policy picks (2D heat, zero and periodic; Bratu's V_k-storing
    # launches; 3D G_Euler! except the V_1 step) -- judged by the instantiation that RAN: the profile
    # names it (the F0R template flag is its last argument) and the library counts FD launches by it;
    # the byte model follows the same instantiation (8 B/pt less exactly where F0R ran)
    jv = [k for k in p0 if k.startswith("jv_fd")]
    assert jv
    if nz:
        uses = lambda k: name == "euler" and k != "jv_fd_dot_v1"  # noqa: E731
    elif name == "bratu2d":  # the V_k-storing launches only
        uses = lambda k: k in ("jv_fd_dot_norm", "jv_fd_dot_v1")  # noqa: E731
    else:
        uses = lambda k: True  # noqa: E731
    stencil = "k_st3l" if nz else "k_st2d"
    # template arguments: k_st2d<KIND, MODE, EPI, VEC, PER, F0R> / k_st3l<KIND, MODE, EPI, VEC, PER, NW, F0R>
    f0r_pos = 6 if nz else 5

    def targs(name):
        return name[name.index("<") + 1:name.rindex(">")].split(", ")
    n_jv = sum(p0[k]["launches"] for k in jv)
    assert p0["_ran"] == {"jv_fd_f0r": 0, "jv_fd_f0_read": n_jv}
    assert p1["_ran"] == {"jv_fd_f0r": sum(p1[k]["launches"] for k in jv if uses(k)),
                          "jv_fd_f0_read": sum(p1[k]["launches"] for k in jv if not uses(k))}
    for k in jv:
        k0, k1 = p0[k]["kernel"], p1[k]["kernel"]
        assert k0.startswith(f"nk::{stencil}<") and targs(k0)[f0r_pos] == "false", (k, k0)
        assert k1.startswith(f"nk::{stencil}<") and targs(k1)[f0r_pos] == ("true" if uses(k) else "false"), (k, k1)
        assert targs(k1)[4] == ("true" if bc == "periodic" else "false"), (k, k1)
        saved = (p0[k]["bytes"] - p1[k]["bytes"]) / p0[k]["timed"] / (8.0 * nx * ny * max(nz, 1))
        assert saved == pytest.approx(1.0 if uses(k) else 0.0, abs=1e-12), (k, saved)


def test_newton_uses_it_and_matches_oracle(ctx):
    """newton_krylov_ passes the flag (res is F(u)); the FD Newton solve still matches the oracle."""
    P = oc.bratu2d(48, 40)
    u0 = oc.sin_ic(P)
    ref, so = oc.newton_krylov(P, u0, jv="fd", memory=20)
    u, r = ah.newton_krylov_(ah.bratu2d_, ah.DeviceArray.from_numpy(u0), (P.hx, P.hy, P.lam), jv="fd", memory=20)
    assert r.solved and so["solved"]
    assert (r.stats.outer_iterations, r.stats.inner_iterations) == (so["outer_iterations"], so["inner_iterations"])
    np.testing.assert_allclose(u.to_numpy(), ref, rtol=0, atol=1e-8 * np.abs(ref).max())
    oc.set_devred(True)  # F(u) recomputed or read, the same bits: the device-order oracle's root
    try:
        ref_dev, _ = oc.newton_krylov(P, u0, jv="fd", memory=20)
    finally:
        oc.set_devred(False)
    np.testing.assert_array_equal(u.to_numpy(), ref_dev)


BRATU_CHILD = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + "/tests")
import _nkpath
import ariadne_hip as ah
from oracle import oracle as oc
import test_hip_f0r as t
ctx = ah.Context(0); ah.set_default_context(ctx)
out = []
for name, nx, ny, bc, nz in [("bratu2d", 200, 150, "zero", 0), ("bratu2d", 201, 37, "zero", 0)] + t.CASES3:
    F, p, u0 = t.case(name, nx, ny, bc, nz)
    kw = dict(restart=True, memory=10, itmax=35, atol=0.0, rtol=0.0)
    x0, h0, n0, p0 = t.solve(F, p, u0, False, **kw)
    x1, h1, n1, p1 = t.solve(F, p, u0, True, **kw)
    jv = [k for k in p0 if k.startswith("jv_fd")]
    assert p1["_ran"]["jv_fd_f0_read"] == 0 and p1["_ran"]["jv_fd_f0r"] == sum(p1[k]["launches"] for k in jv)
    db = sum(p0[k]["bytes"] / p0[k]["timed"] * p0[k]["launches"] - p1[k]["bytes"] / p1[k]["timed"] * p1[k]["launches"] for k in jv)
    out.append(dict(same=bool(h0 == h1 and np.array_equal(x0, x1)), n=int(n1),
                    db=db / (8.0 * nx * ny * max(nz, 1) * sum(p0[k]["launches"] for k in jv))))
print(json.dumps(out))
"""


def test_f0_recomputed_bitwise_when_forced():
    """Every F0R kernel the default policy does not pick -- Bratu 2D, the 3D midpoint / trapezoid and
    V_1 steps -- forced with NK_F0R=2 (a tuning knob of the kernel-variant bench build,
    lib/libnkhip_kbench.so, in a child process: the knob is read once per process)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", BRATU_CHILD, root], env=dict(os.environ, NK_F0R="2", NK_KBENCH_LIB="1"),
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    for r in res:
        assert r["same"] and r["n"] == 35 and r["db"] == pytest.approx(1.0, rel=1e-12)
