"""Implicit time stepping on the HIP path -- examples/implicit.jl.

`solve(G_Euler_, diffusion_, uₙ, p, Δt, ts)` mirrors `solve(G!, f!, uₙ, p, Δt, ts; …)`
(implicit.jl:54-78): one `newton_krylov_` per time step with tol_abs = 6e-6, warn-and-march-on
when a step fails, `uₙ .= u` after each step.  Each composition G! ∘ diffusion! of the three
schemes (G_Euler!, G_Midpoint! with its α keyword, G_Trapezoid!; implicit.jl:8-37) is one fused
device residual (problems._Heat), with bc_zero_ or bc_periodic_ (heat_2D.jl:15-38) in p.
"""
from __future__ import annotations

import logging

from .ariadne import newton_krylov_
from .device import DeviceArray
from .krylov import KrylovConstructor, kcopy_, krylov_workspace
from .problems import _Heat

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
    """G_Euler! / G_Midpoint! / G_Trapezoid! (implicit.jl:8-37) as markers: `bind(f)` returns the fused
    device residual of G ∘ f.  `G_Midpoint_(alpha=…)` is G_Midpoint!'s keyword (default 0.5)."""

    def __init__(self, name, alpha=0.5):
        self.name = name
        self.alpha = float(alpha)

    def __call__(self, *, alpha):
        if self.name != "G_Midpoint!":
            raise TypeError(f"{self.name} takes no keywords")
        return _Scheme(self.name, alpha)

    def bind(self, f):
        if not isinstance(f, _Diffusion):
            raise NotImplementedError(f"no fused device residual for {self.name} ∘ {f}")
        return _Heat(f.dim, self.name, self.alpha)

    def __repr__(self):
        return self.name if self.alpha == 0.5 else f"{self.name}(α = {self.alpha})"


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
