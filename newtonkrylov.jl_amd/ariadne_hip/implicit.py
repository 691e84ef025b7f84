"""Implicit time stepping on the HIP path -- examples/implicit.jl.

`solve(G_Euler_, diffusion_, uₙ, p, Δt, ts)` mirrors `solve(G!, f!, uₙ, p, Δt, ts; …)`
(implicit.jl:54-78): one `newton_krylov_` per time step with tol_abs = 6e-6, warn-and-march-on
when a step fails, `uₙ .= u` after each step.  The composition G_Euler! ∘ diffusion! is one
fused device residual (heat2d_euler_ / heat3d_euler_).  G_Midpoint!/G_Trapezoid! and periodic
boundaries are SURVEY.md §8f "next" items and raise NotImplementedError.
"""
from __future__ import annotations

import logging

from .ariadne import newton_krylov_
from .device import DeviceArray
from .krylov import KrylovConstructor, kcopy_, krylov_workspace
from .problems import heat2d_euler_, heat3d_euler_

log = logging.getLogger("ariadne_hip")


class _Diffusion:
    """diffusion!(du, u, (a, Δx, Δy[, Δz], bc!), t) -- heat_2D.jl:45-62 (marker: fused into G_Euler_)."""

    def __init__(self, dim):
        self.dim = dim

    def __repr__(self):
        return f"diffusion{self.dim}d!"


diffusion_ = _Diffusion(2)
diffusion3d_ = _Diffusion(3)


class _Scheme:
    def __init__(self, name):
        self.name = name

    def bind(self, f):
        if self.name != "G_Euler!":
            raise NotImplementedError(f"{self.name} on the device is a SURVEY.md §8f 'next' item")
        if f is diffusion_:
            return heat2d_euler_
        if f is diffusion3d_:
            return heat3d_euler_
        raise NotImplementedError(f"no fused device residual for {self.name} ∘ {f}")

    def __repr__(self):
        return self.name


G_Euler_ = _Scheme("G_Euler!")
G_Midpoint_ = _Scheme("G_Midpoint!")
G_Trapezoid_ = _Scheme("G_Trapezoid!")


def solve(G_, f_, un: DeviceArray, p, dt: float, ts, *, callback=None, verbose=0, algo="gmres",
          krylov_kwargs=None, memory=20, jv="exact", stats_out=None):
    """Non-adaptive implicit time stepping (implicit.jl:54-78).  Returns uₙ (updated in place)."""
    F_ = G_.bind(f_)
    callback = callback or (lambda u: None)
    u = un.copy()
    du = un.zero()  # temporary of the reference; the fused kernel does not need it
    res = un.zero()
    ws = krylov_workspace(algo, KrylovConstructor(res, memory=memory))  # allocated once, not per step
    ts = list(ts)
    for t in ts[1:]:  # `if t == first(ts) continue`
        _, result = newton_krylov_(F_, u, (un, dt, du, p, t), res, verbose=verbose, algo=algo, tol_abs=6.0e-6,
                                   krylov_kwargs=krylov_kwargs, memory=memory, jv=jv, workspace=ws)
        if stats_out is not None:
            stats_out.append(result)
        if not result.solved:
            log.warning("non linear solve failed marching on t=%s stats=%s", t, result.stats)
        callback(u)
        kcopy_(len(un), un, u)  # uₙ .= u
    ws.free()
    return un
