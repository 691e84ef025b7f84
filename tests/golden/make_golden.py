"""Generate the golden fixtures in tests/golden/ (committed; re-run to regenerate).

Independent of the C oracle: every residual / JVP here is a vectorised numpy restatement
(array slicing, zero padding), Jacobians are assembled as scipy sparse matrices and roots
come from a sparse-direct Newton iteration.  Inputs follow the reference examples:
  * 1D Bratu, N=1000, lambda=3.51382, dx=1/(N+1), u0=sin(pi x)     examples/bratu.jl:40-46
    + the analytic solution true_sol_bratu                          examples/bratu.jl:33-37
  * 2D Bratu (build-defined generalisation), 64^2
  * 2D heat + implicit Euler, N=M=40, a=0.01, explicit-limit dt,   examples/heat_2D.jl:64-91
    reference IC sin(pi x) sin(pi y) on 0:dx:1 (interior part)     + examples/implicit.jl:8-13
  * 3D heat (build-defined), 12^3
  * the 2x2 Kelley system's known answers                           test/runtests.jl:4-46
The reference (Julia) cannot run here (no Julia toolchain), so these fixtures,
plus the known answers transcribed from the reference's tests, are what pins the oracle.

Usage: python tests/golden/make_golden.py
"""
import json
import math
import os

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

HERE = os.path.dirname(os.path.abspath(__file__))
LAM = 3.51382


def lap1d(n, h):
    return sp.diags([np.ones(n - 1), -2.0 * np.ones(n), np.ones(n - 1)], [-1, 0, 1]) / (h * h)


def d2(u, axis, h):
    """((u_+ - 2u) + u_-)/(h*h) with zero Dirichlet (reference evaluation order)."""
    pad = [(0, 0)] * u.ndim
    pad[axis] = (1, 1)
    up = np.pad(u, pad)
    sl = lambda a, b: tuple(slice(a, b) if ax == axis else slice(None) for ax in range(u.ndim))
    n = u.shape[axis]
    return ((up[sl(2, n + 2)] - 2.0 * u) + up[sl(0, n)]) / (h * h)


def newton_sparse(F, J, u, tol=1e-11, maxit=50):
    hist = []
    for _ in range(maxit):
        r = F(u)
        hist.append(float(np.linalg.norm(r)))
        if hist[-1] < tol:
            break
        u = u - spla.spsolve(J(u).tocsc(), r.ravel()).reshape(u.shape)
    return u, hist


def bratu1d():
    N = 1000
    dx = 1.0 / (N + 1)
    x = np.linspace(dx, 1.0 - dx, N)
    u0 = np.sin(x * np.pi)
    F = lambda u: d2(u, 0, dx) + LAM * np.exp(u)
    J = lambda u: lap1d(N, dx) + sp.diags(LAM * np.exp(u))
    rng = np.random.default_rng(1)
    v = rng.standard_normal(N)
    ustar, hist = newton_sparse(F, J, u0.copy())
    theta = 4.79173
    true_sol = -2.0 * np.log(np.cosh(theta * (x - 0.5) / 2.0) / np.cosh(theta / 4.0))
    np.savez_compressed(os.path.join(HERE, "bratu1d_n1000.npz"), x=x, u0=u0, F0=F(u0), v=v,
                        Jv=d2(v, 0, dx) + LAM * (np.exp(u0) * v), ustar=ustar, Fstar_norm=hist[-1],
                        true_sol=true_sol, dx=dx, lam=LAM)


def bratu2d(n=64):
    h = 1.0 / (n + 1)
    xs = np.arange(1, n + 1) * h
    u0 = np.sin(np.pi * xs)[:, None] * np.sin(np.pi * xs)[None, :]
    F = lambda u: (d2(u, 1, h) + d2(u, 0, h)) + LAM * np.exp(u)
    L = sp.kronsum(lap1d(n, h), lap1d(n, h))
    J = lambda u: L + sp.diags(LAM * np.exp(u.ravel()))
    rng = np.random.default_rng(2)
    v = rng.standard_normal((n, n))
    ustar, hist = newton_sparse(F, J, u0.copy())
    np.savez_compressed(os.path.join(HERE, f"bratu2d_{n}.npz"), u0=u0, F0=F(u0), v=v,
                        Jv=(d2(v, 1, h) + d2(v, 0, h)) + LAM * (np.exp(u0) * v), ustar=ustar,
                        Fstar_norm=hist[-1], h=h, lam=LAM)


def heat2d(N=40):
    a = 0.01
    dx = dy = 1.0 / (N + 1)
    dt = dx ** 2 * dy ** 2 / (2.0 * a * (dx ** 2 + dy ** 2))  # heat_2D.jl:72
    xs = np.arange(0, N + 2) * dx                                # 0:Δx:1 (heat_2D.jl:80)
    full = np.sin(np.pi * xs)[:, None] * np.sin(np.pi * xs)[None, :]
    u0 = np.ascontiguousarray(full[1:-1, 1:-1])                  # interior; bc_zero! zeroes the rest
    du = lambda u: a * (d2(u, 1, dx) + d2(u, 0, dy))
    G = lambda u, un: (un + dt * du(u)) - u
    rng = np.random.default_rng(3)
    v = rng.standard_normal((N, N))
    Jv = dt * (a * (d2(v, 1, dx) + d2(v, 0, dy))) - v
    # one exact implicit-Euler step from the eigenvector IC: u1 = u0 / (1 + dt*a*mu)
    mu = 2 * (4.0 / dx ** 2) * math.sin(math.pi * dx / 2) ** 2   # -eigenvalue of the 2D discrete Laplacian
    L = sp.kronsum(lap1d(N, dx), lap1d(N, dy))
    A = (sp.eye(N * N) - dt * a * L).tocsc()
    u1 = spla.spsolve(A, u0.ravel()).reshape(N, N)
    np.savez_compressed(os.path.join(HERE, "heat2d_40.npz"), u0=u0, G0=G(u0, u0), v=v, Jv=Jv, u1=u1,
                        decay=1.0 / (1.0 + dt * a * mu), a=a, dx=dx, dt=dt)


def heat3d(N=12):
    a = 0.01
    h = 1.0 / (N + 1)
    dt = 1.0 / (2.0 * a * (3.0 / h ** 2))
    rng = np.random.default_rng(4)
    xs = np.arange(1, N + 1) * h
    s = np.sin(np.pi * xs)
    u0 = s[:, None, None] * s[None, :, None] * s[None, None, :] + 0.1 * rng.uniform(-1, 1, (N, N, N))
    un = u0.copy()
    u = u0 + 0.01 * rng.standard_normal((N, N, N))
    v = rng.standard_normal((N, N, N))
    du = lambda w: a * ((d2(w, 2, h) + d2(w, 1, h)) + d2(w, 0, h))
    G = (un + dt * du(u)) - u
    Jv = dt * du(v) - v
    np.savez_compressed(os.path.join(HERE, "heat3d_12.npz"), un=un, u=u, G=G, v=v, Jv=Jv, a=a, h=h, dt=dt)


def kelley():
    e2 = math.exp(2.0)
    data = {
        "source": "test/runtests.jl:4-54 (transcribed known answers)",
        "x_jvp": [3.0, 5.0],
        "jvp_e1": [6.0, 7.38905609893065],          # runtests.jl:36-38 (exact equality)
        "vjp_e1": [6.0, 10.0],                      # runtests.jl:40-42
        "jacobian": [[6.0, 10.0], [e2, 10.0]],     # collect(J) == jacobian(Forward, ...) :44-46
        "starts_inplace": [[2.0, 0.5]],             # runtests.jl:15-18, stats.solved
        "starts_outofplace": [[3.0, 5.0]],          # runtests.jl:20-23, stats.solved
        "root": [1.0, 1.0],
    }
    with open(os.path.join(HERE, "kelley2x2.json"), "w") as f:
        json.dump(data, f, indent=1)


if __name__ == "__main__":
    kelley()
    bratu1d()
    bratu2d(64)
    heat2d(40)
    heat3d(12)
    print("goldens written to", HERE)
