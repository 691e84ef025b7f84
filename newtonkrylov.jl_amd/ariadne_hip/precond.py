"""Preconditioners for the device GMRES / FGMRES / CG: Krylov.jl's right `N` and left `M` (ldiv =
false: z = P v approximates J^{-1} v; for CG, M is the SPD preconditioner).  SURVEY.md §8f rank 3:
device Jacobi and ILU(0) preconditioners built from the Jacobian, an inner GMRES, and any other
preconditioner supplied as device code (UserPreconditioner).

`newton_krylov_(…, N=factory, M=factory)`: a factory is called as `factory(J)` once per Newton step
(the JacobianOperator of that step) and returns one of these (e.g. `N=jacobi`, `M=ilu0`).
"""
from __future__ import annotations

import sys

from . import _lib
from ._lib import load
from .device import DeviceArray


class Preconditioner:
    """Base: `as_c()` returns the nk_precond descriptor (kept alive by the object)."""

    def as_c(self) -> _lib.nk_precond:
        raise NotImplementedError

    def apply(self, J, v: DeviceArray, z: DeviceArray | None = None) -> DeviceArray:
        """z = N v (Krylov.jl's mulorldiv!(z, N, v, ldiv)); J = the JacobianOperator a GMRES
        preconditioner solves with (its u / F0 / Jv mode)."""
        import ctypes as C

        z = v.zero() if z is None else z
        prob = J.problem()
        F0 = J.res.ptr if J.jv_mode == _lib.NK_JV_FD else None
        v.ctx.check(load().nk_precond_apply(v.ctx.handle, C.byref(prob), C.byref(self.as_c()), J.u.ptr, F0,
                                            J.jv_mode, z.ptr, v.ptr), "mul!(z, N, v)")
        return z


class DiagonalPreconditioner(Preconditioner):
    """z = d .* v with a device grid function d (NK_PRECOND_DIAG)."""

    def __init__(self, d: DeviceArray):
        self.d = d
        self._c = _lib.nk_precond(_lib.NK_PRECOND_DIAG, d.ptr, _lib.NK_USER_PRECOND(), None)

    def as_c(self):
        return self._c


class UserPreconditioner(Preconditioner):
    """z = N v computed by `apply(z, v)` on DeviceArray views, on the library's stream (runs inside
    ctx.torch_stream() when torch is loaded, like a UserResidual)."""

    def __init__(self, apply, grid, ctx):
        self.apply, self.grid, self.ctx = apply, grid, ctx

        def run(_d, _c, out, inp):
            try:
                o, i = DeviceArray(grid, ctx, _ptr=out), DeviceArray(grid, ctx, _ptr=inp)
                if "torch" in sys.modules:
                    with ctx.torch_stream():
                        apply(o, i)
                else:
                    apply(o, i)
                return 0
            except BaseException as e:
                _lib.set_user_error(e)
                return 1

        self._cb = _lib.NK_USER_PRECOND(run)
        self._c = _lib.nk_precond(_lib.NK_PRECOND_USER, None, self._cb, None)

    def as_c(self):
        return self._c


def jacobian_diag(J, reciprocal: bool = False) -> DeviceArray:
    """diag(J(u)) of a built-in residual on the device (bit-identical to the diagonal of collect(J))."""
    import ctypes as C

    out = J.u.zero()
    prob = J.problem()
    J.u.ctx.check(load().nk_jacobian_diag(J.u.ctx.handle, C.byref(prob), out.ptr, J.u.ptr, int(bool(reciprocal))),
                  "nk_jacobian_diag")
    return out


def jacobi(J) -> DiagonalPreconditioner:
    """Jacobi preconditioner N = diag(J(u))^{-1} (the reference's examples build theirs from
    collect(J), bratu.jl:121-137); use as `N=jacobi` in newton_krylov_ (called per Newton step)."""
    return DiagonalPreconditioner(jacobian_diag(J, reciprocal=True))


class GmresPreconditioner(Preconditioner):
    """`GmresPreconditioner(J, itmax)` of examples/bratu.jl:139-157: mul!(y, P, x) runs
    `gmres(P.J, x; P.itmax)` (Krylov.jl defaults: memory 20, no restart, atol = rtol = √eps) and copies
    the solution into y.  Here the inner solve is the device GMRES on J's operator (NK_PRECOND_GMRES),
    in a workspace of its own; use it with algo="fgmres" (N changes from step to step)."""

    def __init__(self, J, itmax: int, workspace=None):
        from .krylov import KrylovConstructor, krylov_workspace

        self.J, self.itmax = J, int(itmax)
        self.ws = workspace or krylov_workspace("gmres", KrylovConstructor(J.u, memory=20))
        self._c = _lib.nk_precond(_lib.NK_PRECOND_GMRES, None, _lib.NK_USER_PRECOND(), None, self.ws.handle, self.itmax)

    def as_c(self):
        return self._c


def gmres_preconditioner(itmax: int):
    """N factory `(J) -> GmresPreconditioner(J, itmax)` for newton_krylov_ (bratu.jl:150-155); the
    inner workspace is allocated once and reused by every Newton step."""
    cache = {}

    def factory(J):
        key = (id(J.u.ctx), J.u.grid)
        if key not in cache:
            cache.clear()
            cache[key] = GmresPreconditioner(J, itmax).ws
        return GmresPreconditioner(J, itmax, workspace=cache[key])

    return factory


class Ilu0Preconditioner(Preconditioner):
    """`ilu(collect(J))` (examples/bratu.jl:119-137, used with krylov_kwargs = (; ldiv = true)) on the
    device: ILU(0) of J(u) in natural order on J's own sparsity pattern -- for the 1D Bratu Jacobian
    (tridiagonal) this is its exact LU, as IncompleteLU.jl's threshold ILU is there.  Factored once
    (nk_ilu0_factor), applied as z = (L U)^-1 v by two wavefront sweeps (NK_PRECOND_ILU0).  A
    factorisation: it is applied by division, so ldiv=True is accepted (and implied)."""

    ldiv = True

    def __init__(self, J):
        import ctypes as C

        self.J = J
        self.d = J.u.zero()
        prob = J.problem()
        J.u.ctx.check(load().nk_ilu0_factor(J.u.ctx.handle, C.byref(prob), J.u.ptr, self.d.ptr), "nk_ilu0_factor")
        self._c = _lib.nk_precond(_lib.NK_PRECOND_ILU0, self.d.ptr, _lib.NK_USER_PRECOND(), None, None, 0)

    def as_c(self):
        return self._c


def ilu0(J) -> Ilu0Preconditioner:
    """N factory: `N = ilu0` is the device counterpart of `N = (J) -> ilu(collect(J))`."""
    return Ilu0Preconditioner(J)
