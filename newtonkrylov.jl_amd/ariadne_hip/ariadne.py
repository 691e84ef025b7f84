"""Host mirror of Ariadne's public API (src/Ariadne.jl) on the HIP path.

Same names (Julia `!` -> trailing `_`), same keyword arguments and defaults, same control flow
and the same error behaviour (non-finite residual -> log + break, `solved = n_res <= tol`).
The Newton loop is host code, as in the reference; every O(n) operation it triggers runs in
libnkhip.so: the residual stencil, the fused Jv kernel and the device-resident Krylov solve.
"""
from __future__ import annotations

import ctypes as C
import logging
import math
import time
from dataclasses import dataclass
from typing import NamedTuple

from . import _lib
from ._lib import load
from .device import DeviceArray
from .krylov import KrylovConstructor, krylov_solve_, krylov_workspace
from .problems import DeviceResidual, UserResidual

log = logging.getLogger("ariadne_hip")


# ----------------------------------------------------------------------------- forcing (Ariadne.jl:180-217)
class Forcing:
    """Forcing term η of the inexact Newton condition ‖F′(u)d + F(u)‖ <= η ‖F(u)‖."""


@dataclass(frozen=True)
class Fixed(Forcing):
    """Fixed(η = 0.1) -- src/Ariadne.jl:185-192."""
    eta: float = 0.1

    def __call__(self, *args):
        return self.eta

    def initial(self):
        return self.eta


@dataclass(frozen=True)
class EisenstatWalker(Forcing):
    """EisenstatWalker(η_max = 0.999, γ = 0.9) -- src/Ariadne.jl:197-217."""
    eta_max: float = 0.999
    gamma: float = 0.9

    def __call__(self, eta, tol, n_res, n_res_prior):
        eta_res = self.gamma * n_res ** 2 / n_res_prior ** 2
        # Eq 3.6; `γ η^2 <= 1 // 10` is an exact rational comparison, i.e. `< 0.1` for a double
        if self.gamma * eta ** 2 < 0.1:
            eta_safe = min(self.eta_max, eta_res)
        else:
            eta_safe = min(self.eta_max, max(eta_res, self.gamma * eta ** 2))
        return min(self.eta_max, max(eta_safe, 0.5 * tol / n_res))  # Eq 3.5

    def initial(self):
        return self.eta_max


# ----------------------------------------------------------------------------- Jacobian operator
class JacobianOperator:
    """JacobianOperator(F!, res, u, p) -- src/Ariadne.jl:34-46.

    Holds (F, res, u, p) by reference like the reference.  `mul_(out, J, v)` is the device Jv:
    jv="exact" is the dual-number tangent of F (the value Enzyme's forward mode computes in the
    reference's mul!), jv="fd" the north-star operator (F(u + ε v) - F(u)) / ε with F(u) = res.
    """

    def __init__(self, f: DeviceResidual, res: DeviceArray, u: DeviceArray, p=None, jv: str = "exact"):
        if not isinstance(f, DeviceResidual):
            raise TypeError("the HIP JacobianOperator needs a device residual (ariadne_hip.problems); "
                            "generic Python callables have no kernel")
        if jv not in ("exact", "fd"):
            raise ValueError("jv must be 'exact' or 'fd'")
        if jv == "exact" and getattr(f, "J", True) is None:
            raise ValueError(f"{f}: a UserResidual without a tangent J has only the FD operator -- pass jv='fd'")
        self.f, self.res, self.u, self.p = f, res, u, p
        self.jv = jv

    @property
    def jv_mode(self) -> int:
        return _lib.NK_JV_FD if self.jv == "fd" else _lib.NK_JV_EXACT

    def problem(self) -> _lib.nk_problem:
        return self.f.problem(self.u, self.p)

    @property
    def size(self):
        return (len(self.res), len(self.u))

    @property
    def eltype(self):
        return float

    def __len__(self):
        return self.size[0] * self.size[1]


class TransposeOperator:
    """transpose(J) / J' of a JacobianOperator (src/Ariadne.jl:87-107): mul_ gives J(u)^T v."""

    def __init__(self, J: JacobianOperator):
        self.J = J

    @property
    def size(self):
        return tuple(reversed(self.J.size))

    def problem(self) -> _lib.nk_problem:
        return self.J.problem()


def transpose(J: JacobianOperator) -> TransposeOperator:
    return TransposeOperator(J)


JacobianOperator.T = property(transpose)


def mul_(out, J, v, eps: float = 0.0):
    """mul!(out, J, v) (src/Ariadne.jl:48-57); mul!(out, transpose(J), v) (:87-107).  Unlike Enzyme
    it does not rewrite J.res.  Lists of vectors are the batched form mul!(Out, J, V) (:59-85,
    :109-138): ONE fused launch per 8 columns (nk_jv_batched: u, F(u) read once for all of them),
    each column bit-identical to the single-vector product."""
    if isinstance(out, (list, tuple)):
        if not isinstance(v, (list, tuple)) or len(out) != len(v):
            raise ValueError("batched mul!: out and v must be lists of equal length")
        if not out:
            return None
        k = len(out)
        outs = (C.c_void_p * k)(*[o.ptr for o in out])
        vs = (C.c_void_p * k)(*[w.ptr for w in v])
        ctx = out[0].ctx
        if isinstance(J, TransposeOperator):
            prob = J.problem()
            ctx.check(load().nk_jtv_batched(ctx.handle, C.byref(prob), k, outs, J.J.u.ptr, vs), "mul!(Out, J', V)")
            return None
        prob = J.problem()
        F0 = J.res.ptr if J.jv_mode == _lib.NK_JV_FD else None
        ctx.check(load().nk_jv_batched(ctx.handle, C.byref(prob), k, outs, J.u.ptr, vs, F0, J.jv_mode, float(eps)),
                  "mul!(Out, J, V)")
        return None
    if isinstance(J, TransposeOperator):
        prob = J.problem()
        out.ctx.check(load().nk_jtv(out.ctx.handle, C.byref(prob), out.ptr, J.J.u.ptr, v.ptr), "mul!(out, J', v)")
        return None
    prob = J.problem()
    F0 = J.res.ptr if J.jv_mode == _lib.NK_JV_FD else None
    out.ctx.check(load().nk_jv(out.ctx.handle, C.byref(prob), out.ptr, J.u.ptr, v.ptr, F0, J.jv_mode, float(eps)),
                  "mul!(out, J, v)")
    return None


def collect(J, *, coloring: str | None = None):
    """collect(J) (src/Ariadne.jl:140-162): the exact Jacobian J(u) as a scipy.sparse CSC matrix
    (row/column index = interior point in memory order, x fastest; exact zeros dropped like the
    reference's `if out[i] != 0`).  Assembled on the device by nk_jacobian_collect: the built-in
    stencils are probed with 2 dim + 1 coloured vectors in ONE batched launch (a distance-2
    colouring: every probe entry is exactly one Jacobian entry, computed by the same kernel from the
    same operands as the unit-vector probe, so the values are identical), and the CSC arrays are
    written by device kernels; user residuals and periodic grids the colouring does not fit are
    probed with unit vectors, as the reference does.  transpose(J) gives the transpose.  The entries
    are the exact tangent's (Enzyme's mul! in the reference) whatever J's jv mode.
    coloring="dense": unit-vector probing through mul_ from the host (an independent cross-check)."""
    import numpy as np
    import scipy.sparse as sp

    transposed = isinstance(J, TransposeOperator)
    Jo = J.J if transposed else J
    grid = Jo.u.grid
    if Jo.u.ctx.nranks > 1:
        raise NotImplementedError("collect(J) of a distributed operator: gather the slabs first")
    n = grid.n
    if coloring == "dense":
        if n > 4096:
            raise ValueError(f"dense collect(J) probes n = {n} unit vectors from the host; use the default")
        Jx = JacobianOperator(Jo.f, Jo.res, Jo.u, Jo.p, jv="exact")
        Jp = TransposeOperator(Jx) if transposed else Jx
        out = Jo.u.zero()
        cols = []
        e = np.zeros(n)
        for j in range(n):
            e[j] = 1.0
            mul_(out, Jp, DeviceArray.from_numpy(e.reshape(grid.np_shape), grid, Jo.u.ctx))
            e[j] = 0.0
            cols.append(sp.csc_matrix(out.to_numpy().reshape(n, 1)))
        return sp.hstack(cols, format="csc")
    if coloring not in (None, "stencil"):
        raise ValueError("coloring must be 'stencil' (default) or 'dense'")
    prob = Jo.problem()
    user = getattr(Jo.f, "kind", 0) >= _lib.NK_USER1D
    # (2 dim + 1) n bounds a stencil's entries; a user residual's coupling is unknown: retry with nnz
    cap = (2 * grid.dim + 1) * n if not user else min(n * n, 64 * n)
    colptr = np.zeros(n + 1, dtype=np.int64)
    P64 = C.POINTER(C.c_int64)
    nnz = C.c_int64(0)
    for _ in range(2):
        rowval = np.zeros(cap, dtype=np.int64)
        nzval = np.zeros(cap, dtype=np.float64)
        rc = load().nk_jacobian_collect(Jo.u.ctx.handle, C.byref(prob), Jo.u.ptr, int(transposed),
                                        colptr.ctypes.data_as(P64), rowval.ctypes.data_as(P64),
                                        nzval.ctypes.data_as(C.POINTER(C.c_double)), cap, C.byref(nnz))
        if rc == _lib.NK_E_ARG and nnz.value > cap:
            cap = nnz.value
            continue
        Jo.u.ctx.check(rc, "collect(J)")
        break
    m = nnz.value
    return sp.csc_matrix((nzval[:m].copy(), rowval[:m].copy(), colptr), shape=(n, n))


# ----------------------------------------------------------------------------- Newton-Krylov
class Stats(NamedTuple):
    """Stats(outer_iterations, inner_iterations, n_res) -- src/Ariadne.jl:265-276."""
    outer_iterations: int
    inner_iterations: int
    n_res: float

    def update(self, inner_iterations: int, n_res: float) -> "Stats":
        return Stats(self.outer_iterations + 1, self.inner_iterations + inner_iterations, n_res)


class Result(NamedTuple):
    """(; solved, stats, t) -- src/Ariadne.jl:370-371 (+ n_matvec: mul!(J) calls of all Krylov solves)."""
    solved: bool
    stats: Stats
    t: float
    n_matvec: int = 0


def newton_krylov_(F_: DeviceResidual, u: DeviceArray, p=None, res: DeviceArray | None = None, *,
                   tol_rel: float = 1.0e-6, tol_abs: float = 1.0e-12, max_niter: int = 50,
                   forcing: Forcing | None = EisenstatWalker(), verbose: int = 0, algo: str = "gmres",
                   M=None, N=None, krylov_kwargs: dict | None = None, callback=None, memory: int = 20,
                   jv: str = "exact", workspace=None):
    """newton_krylov!(F!, u, p, res; kwargs...) -- src/Ariadne.jl:288-372 (and the 3-arg form :259-263).

    `N` (right) and `M` (left preconditioner) are preconditioner objects or factories `N(J)` /
    `M(J)` called per Newton step (ariadne_hip.precond: `jacobi`, `ilu0`, `gmres_preconditioner`,
    DiagonalPreconditioner, UserPreconditioner), forwarded as Krylov.jl's `N` / `M` (:323-329);
    an `N` or `M` inside krylov_kwargs wins over the factory, as the reference's kwarg merge does.
    Additions of the HIP path: `memory` (Krylov workspace memory = GMRES restart length),
    `jv` ("exact" | "fd") and `workspace` (re-use a Krylov workspace across calls -- the
    reference's own TODO at :316); everything else keeps the reference's meaning and default.
    """
    callback = callback or (lambda *a: None)
    krylov_kwargs = dict(krylov_kwargs or {})
    t0 = time.perf_counter_ns()
    if res is None:
        res = u.zero()  # similar(u₀); Enzyme.make_zero!(res)   (:260-261)
    n = len(u)
    n_res = F_.residual_norm(res, u, p)  # F!(res, u, p); n_res = norm(res)   (:302-303)
    callback(u, res, n_res)

    tol = tol_rel * n_res + tol_abs
    eta = forcing.initial() if forcing is not None else None
    if verbose > 0:
        log.info("Jacobian-Free Newton-Krylov algo=%s res0=%g tol=%g tol_rel=%g tol_abs=%g eta=%s",
                 algo, n_res, tol, tol_rel, tol_abs, eta)

    J = JacobianOperator(F_, res, u, p, jv=jv)
    own_ws = workspace is None
    if own_ws:
        workspace = krylov_workspace(algo, KrylovConstructor(res, memory=memory))
    elif workspace.algo != str(algo).lstrip(":"):
        raise ValueError("workspace algo does not match `algo`")

    stats = Stats(0, 0, n_res)
    n_matvec = 0
    u_norm = 0.0  # ||u|| from the fused update below (the FD step size of the next solve); 0 = unknown
    while n_res > tol and stats.outer_iterations <= max_niter:
        kwargs = dict(krylov_kwargs)
        if forcing is not None:
            kwargs = {"rtol": eta, **kwargs}  # user krylov_kwargs win (:330-333)
        # Solve J d = F(u).  The reference passes copy(res) because Enzyme rewrites res inside
        # mul!; the device operator never writes res, so res itself is the right-hand side.
        # u .-= 1 .* d (Newton step s = 1, :341-344) is fused into the solve's last pass (d =
        # workspace.x is consumed there, not stored), which also returns ||u|| for the next FD step
        # N / M: a preconditioner, or a factory called with this step's operator (e.g. N=jacobi);
        # (; N = N(J), kwargs...), (; M = M(J), kwargs...): the user's krylov_kwargs win (:323-329)
        if N is not None and "N" not in kwargs:
            kwargs["N"] = N if hasattr(N, "as_c") else N(J)
        if M is not None and "M" not in kwargs:
            kwargs["M"] = M if hasattr(M, "as_c") else M(J)
        krylov_solve_(workspace, J, res, _b_norm=n_res, _u_norm=u_norm, _u_update=u, _f0_is_residual=True, **kwargs)
        n_matvec += workspace.stats.n_matvec
        u_norm = workspace.stats.u_norm
        n_res_prior = n_res
        n_res = F_.residual_norm(res, u, p)
        callback(u, res, n_res)
        if math.isinf(n_res) or math.isnan(n_res):
            log.error("Inner solver blew up: %s", stats)
            break
        if forcing is not None:
            eta = forcing(eta, tol, n_res, n_res_prior)
        if verbose > 0 and workspace.stats.niter == 0 and forcing is not None:
            log.info("Inexact Newton thinks our step is good enough eta=%g %s", eta, stats)
        stats = stats.update(workspace.stats.niter, n_res)
        if verbose > 0:
            log.info("Newton iter=%g eta=%s %s", n_res, eta, stats)
    t = (time.perf_counter_ns() - t0) / 1.0e9
    if own_ws:
        workspace.free()
    return u, Result(n_res <= tol, stats, t, n_matvec)


def newton_krylov_native(F_: DeviceResidual, u: DeviceArray, p=None, res: DeviceArray | None = None, *,
                         tol_rel: float = 1.0e-6, tol_abs: float = 1.0e-12, max_niter: int = 50,
                         forcing: Forcing | None = EisenstatWalker(), algo: str = "gmres",
                         krylov_kwargs: dict | None = None, memory: int = 20, jv: str = "exact"):
    """newton_krylov_ with the loop itself in libnkhip.so (nk_newton_krylov, the C/C++ callers' entry
    point).  Same arguments, same result; returns (u, Result) with the histories of ||F||."""
    kk = dict(krylov_kwargs or {})
    unknown = set(kk) - {"restart", "reorthogonalization", "itmax", "atol", "rtol"}
    if unknown:
        raise TypeError(f"unsupported Krylov keyword(s): {sorted(unknown)}")
    if res is None:
        res = u.zero()
    o = _lib.nk_newton_opts()
    load().nk_newton_defaults(C.byref(o))
    o.tol_rel, o.tol_abs, o.max_niter = float(tol_rel), float(tol_abs), int(max_niter)
    if forcing is None:
        o.forcing = _lib.NK_FORCING_NONE
    elif isinstance(forcing, Fixed):
        o.forcing, o.eta = _lib.NK_FORCING_FIXED, float(forcing.eta)
    elif isinstance(forcing, EisenstatWalker):
        o.forcing, o.eta_max, o.gamma = _lib.NK_FORCING_EW, float(forcing.eta_max), float(forcing.gamma)
    else:
        raise TypeError("forcing must be Fixed, EisenstatWalker or None")
    o.algo = {"gmres": _lib.NK_ALGO_GMRES, "cg": _lib.NK_ALGO_CG}[str(algo).lstrip(":")]
    o.memory = int(memory)
    o.krylov.restart = int(bool(kk.get("restart", False)))
    o.krylov.reorthogonalization = int(bool(kk.get("reorthogonalization", False)))
    o.krylov.itmax = int(kk.get("itmax", 0))
    o.krylov.jv_mode = _lib.NK_JV_FD if jv == "fd" else _lib.NK_JV_EXACT
    o.krylov.atol = float(kk.get("atol", o.krylov.atol))
    if "rtol" in kk:
        o.krylov.rtol, o.rtol_user = float(kk["rtol"]), 1
    st = _lib.nk_newton_stats()
    cap = int(max_niter) + 2
    hist = (C.c_double * cap)()
    hl = C.c_int64(0)
    t0 = time.perf_counter_ns()
    prob = F_.problem(u, p)
    u.ctx.check(load().nk_newton_krylov(u.ctx.handle, C.byref(prob), u.ptr, res.ptr, C.byref(o), C.byref(st), hist,
                                        cap, C.byref(hl)), "nk_newton_krylov")
    t = (time.perf_counter_ns() - t0) / 1.0e9
    stats = Stats(int(st.outer_iterations), int(st.inner_iterations), float(st.n_res))
    return u, Result(bool(st.solved), stats, t, int(st.n_matvec))


def newton_krylov(F, u0: DeviceArray, p=None, **kwargs):
    """newton_krylov(F, u₀, p; kwargs...) -- out-of-place form (src/Ariadne.jl:245-248): u₀ is not
    modified.  F is a device residual (in place, as newton_krylov_ takes), or -- the reference's
    out-of-place `F(u, p)` that returns the residual -- a plain callable that gets u as a torch view
    and returns a tensor of u's shape; it is wrapped as F!(res, u, p) = (res .= F(u, p)) (:245-246),
    a user residual without a tangent, so pass jv="fd"."""
    if not isinstance(F, DeviceResidual):
        if not callable(F):
            raise TypeError("newton_krylov: F must be a device residual or a callable F(u, p)")
        fn = F

        def F_inplace(res, u, p_):
            res.torch().copy_(fn(u.torch(), p_).reshape(res.torch().shape))

        F = UserResidual(F_inplace, name=getattr(fn, "__name__", "F") + "!")
    return newton_krylov_(F, u0.copy(), p, **kwargs)
