"""Device residuals: the `F!(res, u, p)` callbacks of the reference examples, as HIP stencils.

A `DeviceResidual` is called exactly like the reference's residual functions, with the same
parameter tuples, but it launches a hand-written gfx950 kernel (nk_residual) instead of a Julia
loop, and `JacobianOperator` maps it to the matching fused Jv kernel (nk_jv) instead of Enzyme.

| object        | reference                                             | p                                   |
|---------------|-------------------------------------------------------|-------------------------------------|
| `bratu_`      | `bratu!(res, y, (Δx, λ))`  examples/bratu.jl:14-24    | `(dx, lam)`                          |
| `bratu2d_`    | 2D generalisation                  | `(dx, dy, lam)`                      |
| `heat2d_euler_` | `G_Euler!` ∘ `diffusion!` implicit.jl:8-13 + heat_2D.jl:45-62 | `(u_n, dt, du, (a, dx, dy, bc_zero_), t)` |
| `heat3d_euler_` | 3D generalisation                | `(u_n, dt, du, (a, dx, dy, dz, bc_zero_), t)` |
| `heat{2,3}d_midpoint_`, `heat{2,3}d_trapezoid_` | `G_Midpoint!` / `G_Trapezoid!` ∘ `diffusion!` implicit.jl:17-37 | as above; `bc_periodic_` (heat_2D.jl:15-26) for any heat residual |
| `UserResidual(F[, J])` | any `F!(res, u, p)` evaluated on the device by the caller | the caller's |
"""
from __future__ import annotations

import ctypes as C
import sys

from . import _lib
from ._lib import load
from .device import DeviceArray


def bc_zero_(u):
    """`bc_zero!` (heat_2D.jl:28-38): zero ghost cells.  DeviceArray ghosts are zero by
    construction (or hold the neighbour slab's plane), so this is a marker, not an action."""
    return None


class DeviceResidual:
    """F!(res, u, p) backed by a HIP stencil kernel."""

    kind: int
    name: str

    def problem(self, u: DeviceArray, p) -> _lib.nk_problem:
        raise NotImplementedError

    def __call__(self, res: DeviceArray, u: DeviceArray, p=None):
        prob = self.problem(u, p)
        u.ctx.check(load().nk_residual(u.ctx.handle, C.byref(prob), res.ptr, u.ptr), f"{self.name}")
        return None

    def residual_norm(self, res: DeviceArray, u: DeviceArray, p=None) -> float:
        """F!(res, u, p); norm(res) as one fused pass (src/Ariadne.jl:302-303, :349-350)."""
        prob = self.problem(u, p)
        out = C.c_double()
        u.ctx.check(load().nk_residual_norm(u.ctx.handle, C.byref(prob), res.ptr, u.ptr, C.byref(out)), self.name)
        return out.value

    def __repr__(self):
        return self.name


class _Bratu1D(DeviceResidual):
    kind, name = _lib.NK_BRATU1D, "bratu!"

    def problem(self, u, p):
        dx, lam = p
        if u.grid.dim != 1:
            raise ValueError("bratu! is the 1D problem")
        nx, ny, nz = u.grid.nxyz
        return _lib.nk_problem(self.kind, 0, nx, 1, 1, float(dx), 1.0, 1.0, float(lam), 0.0, 0.0, None)


class _Bratu2D(DeviceResidual):
    kind, name = _lib.NK_BRATU2D, "bratu2d!"

    def problem(self, u, p):
        dx, dy, lam = p
        if u.grid.dim != 2:
            raise ValueError("bratu2d! needs a 2D grid")
        nx, ny, _ = u.grid.nxyz
        return _lib.nk_problem(self.kind, 0, nx, ny, 1, float(dx), float(dy), 1.0, float(lam), 0.0, 0.0, None)


def bc_periodic_(u):
    """`bc_periodic!` (heat_2D.jl:15-26): a marker.  The kernels wrap x (and y in 3D) and the library
    fills the ghost planes along the slab axis with the opposite edge (a ring exchange when
    distributed) before every stencil, including for the tangent v -- what Enzyme's forward
    mode does to the shadow ghosts."""
    return None


_SCHEMES = {  # implicit.jl:8-37
    ("G_Euler!", 2): _lib.NK_HEAT2D_EULER, ("G_Euler!", 3): _lib.NK_HEAT3D_EULER,
    ("G_Midpoint!", 2): _lib.NK_HEAT2D_MIDPOINT, ("G_Midpoint!", 3): _lib.NK_HEAT3D_MIDPOINT,
    ("G_Trapezoid!", 2): _lib.NK_HEAT2D_TRAPEZOID, ("G_Trapezoid!", 3): _lib.NK_HEAT3D_TRAPEZOID,
}


class _Heat(DeviceResidual):
    """F!(res, u, (uₙ, Δt, du, p, t)) = G!(res, uₙ, Δt, diffusion!, du, u, p, t) for G ∈ {G_Euler!,
    G_Midpoint!(α), G_Trapezoid!} (implicit.jl:8-37, 61), p = (a, Δx, Δy[, Δz], bc!) with bc! one of
    bc_zero_ / bc_periodic_ (heat_2D.jl:15-38).  One fused stencil kernel per call."""

    def __init__(self, dim: int, scheme: str = "G_Euler!", alpha: float = 0.5):
        self.dim, self.scheme, self.alpha = dim, scheme, float(alpha)
        self.kind = _SCHEMES[scheme, dim]
        a = f"(α = {self.alpha})" if scheme == "G_Midpoint!" and self.alpha != 0.5 else ""
        self.name = f"{scheme}{a}∘diffusion{dim}d!"

    def with_alpha(self, alpha: float) -> "_Heat":
        """G_Midpoint!(…; α) -- the keyword of implicit.jl:17."""
        if self.scheme != "G_Midpoint!":
            raise ValueError("α is a G_Midpoint! keyword")
        return _Heat(self.dim, self.scheme, alpha)

    def problem(self, u, p):
        un, dt, _du, fp, _t = p
        if u.grid.dim != self.dim:
            raise ValueError(f"{self.name} needs a {self.dim}D grid")
        if self.dim == 2:
            a, dx, dy, bc = fp
            dz = 1.0
        else:
            a, dx, dy, dz, bc = fp
        if bc is bc_zero_:
            code = _lib.NK_BC_ZERO
        elif bc is bc_periodic_:
            code = _lib.NK_BC_PERIODIC
        else:
            raise NotImplementedError(f"boundary {bc!r}: the device kernels implement bc_zero_ and bc_periodic_")
        if not isinstance(un, DeviceArray) or un.grid != u.grid:
            raise ValueError("u_n must be a DeviceArray on u's grid")
        nx, ny, nz = u.grid.nxyz
        return _lib.nk_problem(self.kind, code, nx, ny, nz, float(dx), float(dy), float(dz), 0.0, float(a), float(dt),
                               un.ptr, None, self.alpha)


_HeatEuler = _Heat  # backwards-compatible name

bratu_ = _Bratu1D()
bratu2d_ = _Bratu2D()
heat2d_euler_ = _Heat(2)
heat3d_euler_ = _Heat(3)
heat2d_midpoint_ = _Heat(2, "G_Midpoint!")
heat3d_midpoint_ = _Heat(3, "G_Midpoint!")
heat2d_trapezoid_ = _Heat(2, "G_Trapezoid!")
heat3d_trapezoid_ = _Heat(3, "G_Trapezoid!")


# ----------------------------------------------------------------------------- user residuals
class UserResidual(DeviceResidual):
    """F!(res, u, p) written by the caller -- the residual callback newton_krylov! takes
    (src/Ariadne.jl:288; e.g. the KernelAbstractions residual of examples/bratu_ka.jl) -- for
    residuals that have no built-in kernel (kinds NK_USER1D/2D/3D).

    `F(res, u, p)` gets DeviceArray views of device vectors on u's grid and must evaluate the
    residual ON THE DEVICE, enqueued on the library's stream: the call already runs inside
    `ctx.torch_stream()` when torch is loaded, so `res.torch()[...] = f(u.torch())` just works.
    Ghost planes of u are current (zero Dirichlet, or the neighbour slab's plane).
    `JT(out, u, v, p)` (optional) is the transpose product J(u)^T v (mul! on transpose(J)).
    `J(out, u, v, p)` (optional) is the exact tangent -- what Enzyme's forward mode computes for the
    reference's mul! (src/Ariadne.jl:48-57); without it use JacobianOperator(..., jv="fd"), whose
    FD quotient, basis normalisation and reductions the library runs around F on the device.
    """

    kind = _lib.NK_USER2D  # per call: NK_USER1D/2D/3D by the grid's dimension

    def __init__(self, F, J=None, name: str | None = None, JT=None):
        self.F, self.J, self.JT = F, J, JT
        self.name = name or (getattr(F, "__name__", "user") + "!")
        self._live = {}

    def _callbacks(self, grid, ctx, p):
        def run(fn, *ptrs):
            try:
                views = [DeviceArray(grid, ctx, _ptr=q) for q in ptrs]
                if "torch" in sys.modules:
                    with ctx.torch_stream():
                        fn(*views, p)
                else:
                    fn(*views, p)
                return 0
            except BaseException as e:  # reported by the C call that invoked the callback
                _lib.set_user_error(e)
                return 1

        cf = _lib.NK_USER_RESIDUAL(lambda _d, _c, res, u: run(self.F, res, u))
        cj = _lib.NK_USER_TANGENT(lambda _d, _c, out, u, v: run(self.J, out, u, v)) if self.J else _lib.NK_USER_TANGENT()
        ct = (_lib.NK_USER_TANGENT(lambda _d, _c, out, u, v: run(self.JT, out, u, v)) if self.JT
              else _lib.NK_USER_TANGENT())
        ops = _lib.nk_user_ops(cf, cj, ct, None)
        return ops, cf, (cj, ct)

    def problem(self, u, p):
        key = (u.grid, id(u.ctx), id(p))
        hit = self._live.get(key)
        if hit is None:
            if len(self._live) > 16:
                self._live.clear()
            ops, cf, cj = self._callbacks(u.grid, u.ctx, p)
            hit = self._live[key] = (ops, cf, cj, p)  # keeps the callbacks (and p) alive
        nx, ny, nz = u.grid.nxyz
        kind = (_lib.NK_USER1D, _lib.NK_USER2D, _lib.NK_USER3D)[u.grid.dim - 1]
        return _lib.nk_problem(kind, 0, nx, ny, nz, 1.0, 1.0, 1.0, 0.0, 0.0, 0.0, None,
                               C.cast(C.pointer(hit[0]), C.c_void_p))
