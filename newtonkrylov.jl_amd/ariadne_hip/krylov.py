"""Krylov.jl's plug-in surface on device vectors.

* vector primitives `kdot, knorm, kscal_, kaxpy_, kaxpby_, kcopy_, kfill_, kdivcopy_, kref_`:
  the overload points `examples/halovector.jl:51-147` implements for HaloVector -- here each is
  one HIP kernel (dot/norm return host scalars, as in Krylov.jl);
* `KrylovConstructor`, `krylov_workspace`, `krylov_solve_`: what Ariadne calls at
  src/Ariadne.jl:317-318 and :338.  The solve runs the device-resident GMRES / CG of
  libnkhip.so (nk_krylov_solve), a restatement of Krylov.jl 0.10.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import load
from .device import DeviceArray

SQRT_EPS = math.sqrt(np.finfo(np.float64).eps)


def _h(x: DeviceArray):
    return x.ctx.handle


# -------------------------------------------------------------------------- vector primitives
def exp_(y, x, ctx=None):
    """y .= exp.(x) with the library's correctly rounded exp (nk_vexp: the exp of the Bratu stencils,
    csrc/nk_exp.h, which the CPU oracle compiles too) -- for user residuals, so that runtests.jl:4-13's
    exp(x1 - 1) evaluates exactly as the oracle's.  y, x: DeviceArrays, or contiguous float64 torch
    tensors on the context's device (enqueued on the library stream, where user callbacks run)."""
    from .device import default_context

    ctx = ctx or (y.ctx if isinstance(y, DeviceArray) else x.ctx if isinstance(x, DeviceArray) else default_context())

    def ptr_len(a, what):
        # every operand must live on THIS context's GPU: a host tensor's (or another device's) address
        # handed to the kernel would fault the GPU instead of raising
        if isinstance(a, DeviceArray):
            if a.ctx is not ctx:
                raise ValueError(f"exp_: {what} belongs to another context")
            return a.ptr, a.n
        if not hasattr(a, "data_ptr"):
            raise ValueError(f"exp_: {what} must be a DeviceArray or a torch tensor")
        if a.dtype != __import__("torch").float64 or not a.is_contiguous():
            raise ValueError("exp_: contiguous float64 tensors only")
        if not a.is_cuda or a.device.index != ctx.device:
            raise ValueError(f"exp_: {what} must be on the context's GPU (cuda:{ctx.device}), not {a.device}")
        return a.data_ptr(), a.numel()

    (py, ny), (px, nx) = ptr_len(y, "y"), ptr_len(x, "x")
    if ny != nx:
        raise ValueError(f"exp_: lengths differ ({ny} vs {nx})")
    ctx.check(load().nk_vexp(ctx.handle, nx, py, px), "nk_vexp")
    return y


def kdot(n: int, x: DeviceArray, y: DeviceArray) -> float:
    out = C.c_double()
    x.ctx.check(load().nk_dot(_h(x), n, x.ptr, y.ptr, C.byref(out)), "kdot")
    return out.value


def knorm(n: int, x: DeviceArray) -> float:
    out = C.c_double()
    x.ctx.check(load().nk_norm(_h(x), n, x.ptr, C.byref(out)), "knorm")
    return out.value


def kscal_(n: int, s: float, x: DeviceArray):
    x.ctx.check(load().nk_scal(_h(x), n, float(s), x.ptr), "kscal!")
    return x


def kaxpy_(n: int, s: float, x: DeviceArray, y: DeviceArray):
    y.ctx.check(load().nk_axpy(_h(y), n, float(s), x.ptr, y.ptr), "kaxpy!")
    return y


def kaxpy_norm_(n: int, s: float, x: DeviceArray, y: DeviceArray) -> float:
    """y = s x + y, returning ||y|| from the same pass (nk_axpy_norm): the Newton update u .-= d
    (src/Ariadne.jl:344) fused with the ||u|| the next FD operator needs."""
    out = C.c_double()
    y.ctx.check(load().nk_axpy_norm(_h(y), n, float(s), x.ptr, y.ptr, C.byref(out)), "kaxpy!")
    return out.value


def kaxpby_(n: int, s: float, x: DeviceArray, t: float, y: DeviceArray):
    y.ctx.check(load().nk_axpby(_h(y), n, float(s), x.ptr, float(t), y.ptr), "kaxpby!")
    return y


def kcopy_(n: int, y: DeviceArray, x: DeviceArray):
    y.ctx.check(load().nk_copy(_h(y), n, y.ptr, x.ptr), "kcopy!")
    return y


def kfill_(x: DeviceArray, val: float):
    x.ctx.check(load().nk_fill(_h(x), x.n, x.ptr, float(val)), "kfill!")
    return x


def kdivcopy_(n: int, y: DeviceArray, x: DeviceArray, s: float):
    y.ctx.check(load().nk_divcopy(_h(y), n, y.ptr, x.ptr, float(s)), "kdivcopy!")
    return y


def kref_(n: int, x: DeviceArray, y: DeviceArray, c: float, s: float):
    x.ctx.check(load().nk_ref(_h(x), n, x.ptr, y.ptr, float(c), float(s)), "kref!")
    return x, y


def mgs_step_(V, q: DeviceArray, reorthogonalization: bool = False):
    """One fused modified-Gram-Schmidt sweep of q against the basis V (Krylov.jl gmres! inner loop):
    q is orthogonalised in place; returns the Hessenberg column [h_1 .. h_k, ||q||] (nk_mgs_step)."""
    k = len(V)
    ptrs = (C.c_void_p * k)(*[v.ptr for v in V])
    h = (C.c_double * (k + 1))()
    q.ctx.check(load().nk_mgs_step(_h(q), len(q), ptrs, k, q.ptr, int(bool(reorthogonalization)), h), "mgs_step!")
    return np.array(h[:])


# -------------------------------------------------------------------------- workspace / solve
@dataclass
class KrylovConstructor:
    """KrylovConstructor(res) (src/Ariadne.jl:317): workspace vectors follow `similar(res)`.

    `memory` is Krylov.jl's workspace argument (default 20).  Ariadne cannot forward it
    (SURVEY.md §8a A1); the host mirror exposes it so GMRES(30) (BASELINE config 2) is expressible.
    """
    vm: DeviceArray
    memory: int = 20


@dataclass
class KrylovStats:
    niter: int = 0
    solved: bool = False
    inconsistent: bool = False
    status: str = "unknown"
    n_matvec: int = 0
    residuals: list = field(default_factory=list)
    u_norm: float = 0.0  # ||u|| after a fused Newton update (_u_update)


_STATUS = {0: "unknown", 1: "solution good enough given atol and rtol", 2: "maximum number of iterations exceeded",
           3: "breakdown", 4: "zero curvature detected"}
_ALGOS = {"gmres": _lib.NK_ALGO_GMRES, "cg": _lib.NK_ALGO_CG, "fgmres": _lib.NK_ALGO_FGMRES}


class KrylovWorkspace:
    """krylov_workspace(algo, kc): device basis + x, allocated once and reused every Newton step."""

    def __init__(self, algo: str, kc: KrylovConstructor):
        if algo not in _ALGOS:
            raise NotImplementedError(f"algo = :{algo} -- the HIP path implements :gmres, :fgmres and :cg "
                                      "(other Krylov methods are out of scope, SURVEY.md §2 C16)")
        self.algo = algo
        self.memory = int(kc.memory)
        self.ctx = kc.vm.ctx
        self.grid = kc.vm.grid
        gp = self.grid.geometry_problem()
        h = C.c_void_p()
        self.ctx.check(load().nk_workspace_create(self.ctx.handle, _ALGOS[algo], C.byref(gp), self.memory, C.byref(h)),
                       "krylov_workspace")
        self.handle = h
        self.x = DeviceArray(self.grid, self.ctx, _ptr=load().nk_workspace_x(h))
        self.stats = KrylovStats()

    def basis(self, i: int) -> DeviceArray | None:
        """workspace.V[i + 1] of the last Arnoldi cycle (a device view; None past the allocated basis)."""
        p = load().nk_workspace_basis(self.handle, int(i))
        return DeviceArray(self.grid, self.ctx, _ptr=p) if p else None

    def free(self):
        if getattr(self, "handle", None) and self.ctx.handle:
            load().nk_workspace_destroy(self.handle)
        self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def krylov_workspace(algo, kc: KrylovConstructor) -> KrylovWorkspace:
    return KrylovWorkspace(str(algo).lstrip(":"), kc)


def krylov_solve_(ws: KrylovWorkspace, J, b: DeviceArray, *, restart=False, reorthogonalization=False,
                  atol=SQRT_EPS, rtol=SQRT_EPS, itmax=0, history=False, verbose=0, M=None, N=None, ldiv=False,
                  _b_norm=0.0, _u_norm=0.0, _u_update=None, _f0_is_residual=False, **unknown):
    """krylov_solve!(workspace, J, b; kwargs...) for a JacobianOperator J on device vectors.
    (_b_norm / _u_norm: norms the Newton loop already holds -- ||F(u)|| and ||u|| -- so the solve
    does not stream b and u once more just to recompute them.  _u_update = u: the Newton update
    u .-= x is fused into the last pass; ws.x is then not stored and ws.stats.u_norm = ||u||.
    _f0_is_residual: J.res is exactly F(u) as the device residual computed it -- the Newton loop's res
    -- so the 2D FD stencils recompute it instead of loading it; bit-identical.)"""
    if unknown:
        raise TypeError(f"unsupported Krylov keyword(s): {sorted(unknown)}")
    for name, P in (("N", N), ("M", M)):
        if ldiv and P is not None and not getattr(P, "ldiv", False):
            raise NotImplementedError(f"ldiv = true: give {name} as the operator that approximates J^{{-1}} "
                                      "(ldiv = false), or a factorisation (ilu0)")
        if P is not None and not hasattr(P, "as_c"):
            raise TypeError(f"{name} must be an ariadne_hip preconditioner (DiagonalPreconditioner, "
                            "UserPreconditioner, GmresPreconditioner, jacobi(J), ilu0(J))")
    if ws.algo == "cg" and N is not None:
        raise TypeError("cg! takes its preconditioner as M (Krylov.jl has no right preconditioner for CG)")
    if ws.algo == "cg" and (restart or reorthogonalization):
        raise TypeError("restart / reorthogonalization are GMRES keywords")
    prob = J.problem()
    opts = _lib.nk_krylov_opts(int(bool(restart)), int(bool(reorthogonalization)), int(itmax), J.jv_mode,
                               float(atol), float(rtol), float(_b_norm), float(_u_norm),
                               _u_update.ptr if _u_update is not None else None,
                               C.cast(C.pointer(N.as_c()), C.c_void_p) if N is not None else None,
                               C.cast(C.pointer(M.as_c()), C.c_void_p) if M is not None else None,
                               int(bool(_f0_is_residual)))
    st = _lib.nk_krylov_stats()
    cap = ((int(itmax) or 4096) + 64) if history else 0
    hist = (C.c_double * max(cap, 1))()
    hl = C.c_int64(0)
    F0 = J.res.ptr if J.jv_mode == _lib.NK_JV_FD else None
    ws.ctx.check(load().nk_krylov_solve(ws.handle, C.byref(prob), J.u.ptr, F0, b.ptr, C.byref(opts), C.byref(st),
                                        hist, cap, C.byref(hl)), "krylov_solve!")
    ws.stats = KrylovStats(niter=int(st.niter), solved=bool(st.solved), inconsistent=bool(st.inconsistent),
                           status=_STATUS.get(st.status, "unknown"), n_matvec=int(st.n_matvec),
                           residuals=list(hist[: min(hl.value, cap)]) if history else [], u_norm=float(st.u_norm))
    if verbose:
        print(f"{ws.algo.upper()}: niter={ws.stats.niter} status={ws.stats.status}")
    return ws
