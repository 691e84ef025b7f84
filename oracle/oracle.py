"""ctypes front-end of the C oracle (oracle/nk_oracle.c).

TEST INFRASTRUCTURE ONLY.  Only tests/, ``__graft_entry__.smoke()`` and bench.py's
``cpu_baseline`` leg may import this module -- as the checker / the timed CPU baseline,
never as the thing measured or shipped.  The product package (newtonkrylov.jl_amd/)
never imports it and has no CPU fallback.

Each function restates the reference (file:line in nk_oracle.c); parity of the
Krylov.jl part (third-party, absent from /root/reference) is pinned only through the
reference's known answers and the numpy/scipy goldens in tests/golden/.
"""
from __future__ import annotations

import ctypes as C
import math
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libnkoracle.so")

BRATU1D, BRATU2D, HEAT2D_EULER, HEAT3D_EULER = 1, 2, 3, 4
HEAT2D_MIDPOINT, HEAT3D_MIDPOINT, HEAT2D_TRAPEZOID, HEAT3D_TRAPEZOID = 5, 6, 7, 8
BC_ZERO, BC_PERIODIC = 0, 1
HEAT_KINDS = {  # (scheme, dim) -> kind; schemes of examples/implicit.jl:8-37
    ("euler", 2): HEAT2D_EULER, ("euler", 3): HEAT3D_EULER,
    ("midpoint", 2): HEAT2D_MIDPOINT, ("midpoint", 3): HEAT3D_MIDPOINT,
    ("trapezoid", 2): HEAT2D_TRAPEZOID, ("trapezoid", 3): HEAT3D_TRAPEZOID,
}
JV_EXACT, JV_FD = 0, 1
FORCING_NONE, FORCING_FIXED, FORCING_EW = 0, 1, 2
ALGO_GMRES, ALGO_CG, ALGO_FGMRES = 0, 1, 2
PRECOND_NONE, PRECOND_DIAG, PRECOND_GMRES, PRECOND_JACOBI, PRECOND_ILU0, PRECOND_ILU = 0, 1, 3, 4, 5, 6
_ALGO = {"gmres": ALGO_GMRES, "cg": ALGO_CG, "fgmres": ALGO_FGMRES}
SQRT_EPS = math.sqrt(np.finfo(np.float64).eps)


class _Problem(C.Structure):
    _fields_ = [("kind", C.c_int32), ("bc", C.c_int32),
                ("nx", C.c_int64), ("ny", C.c_int64), ("nz", C.c_int64),
                ("hx", C.c_double), ("hy", C.c_double), ("hz", C.c_double),
                ("lam", C.c_double), ("a", C.c_double), ("dt", C.c_double),
                ("un", C.POINTER(C.c_double)), ("alpha", C.c_double)]


class _Precond(C.Structure):
    _fields_ = [("kind", C.c_int32), ("itmax", C.c_int32), ("diag", C.POINTER(C.c_double)), ("P", C.c_void_p)]


class _KrylovOpts(C.Structure):
    _fields_ = [("memory", C.c_int32), ("restart", C.c_int32), ("reorthogonalization", C.c_int32),
                ("itmax", C.c_int32), ("atol", C.c_double), ("rtol", C.c_double), ("flexible", C.c_int32),
                ("N", C.POINTER(_Precond)), ("M", C.POINTER(_Precond))]


class _KrylovStats(C.Structure):
    _fields_ = [("niter", C.c_int64), ("solved", C.c_int32), ("inconsistent", C.c_int32),
                ("breakdown", C.c_int32), ("status", C.c_int32), ("n_matvec", C.c_int64)]


class _NewtonOpts(C.Structure):
    _fields_ = [("tol_rel", C.c_double), ("tol_abs", C.c_double), ("max_niter", C.c_int32),
                ("forcing", C.c_int32), ("eta_fixed", C.c_double), ("eta_max", C.c_double),
                ("gamma", C.c_double), ("algo", C.c_int32), ("jv_mode", C.c_int32),
                ("krylov", _KrylovOpts), ("rtol_user", C.c_int32), ("precond", C.c_int32),
                ("precond_itmax", C.c_int32), ("mprecond", C.c_int32), ("mprecond_itmax", C.c_int32)]


class _NewtonStats(C.Structure):
    _fields_ = [("outer_iterations", C.c_int64), ("inner_iterations", C.c_int64), ("n_res", C.c_double),
                ("solved", C.c_int32), ("n_matvec", C.c_int64), ("n_residual", C.c_int64), ("tol", C.c_double)]


_lib = None


# the correctly rounded exp the oracle shares with the HIP stencils (compiled into nk_oracle.c)
EXP_H = os.path.join(os.path.dirname(HERE), "newtonkrylov.jl_amd", "csrc", "nk_exp.h")


def build() -> str:
    """Compile the oracle with its Makefile (gcc is part of the image)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        srcs = (os.path.join(HERE, "nk_oracle.c"), EXP_H)
        if not all(os.path.exists(f) for f in (LIB_PATH, LIBM_PATH)) or any(
                os.path.getmtime(LIB_PATH) < os.path.getmtime(f) for f in srcs if os.path.exists(f)):
            build()
        L = C.CDLL(LIB_PATH)
        D, I64, P = C.c_double, C.c_int64, C.POINTER(C.c_double)
        L.oc_dot.restype = D
        L.oc_dot.argtypes = [I64, P, P]
        L.oc_norm.restype = D
        L.oc_norm.argtypes = [I64, P]
        L.oc_fd_eps.restype = D
        L.oc_fd_eps.argtypes = [D, D]
        L.oc_ew_forcing.restype = D
        L.oc_ew_forcing.argtypes = [D, D, D, D, D, D]
        L.oc_residual.argtypes = [C.POINTER(_Problem), P, P]
        L.oc_jv_exact.argtypes = [C.POINTER(_Problem), P, P, P]
        L.oc_jv_fd.argtypes = [C.POINTER(_Problem), P, P, P, P, D]
        L.oc_krylov_solve.argtypes = [C.POINTER(_Problem), C.c_int, C.c_int, P, P, P, P,
                                      C.POINTER(_KrylovOpts), C.POINTER(_KrylovStats), P, I64, C.POINTER(I64)]
        L.oc_newton_krylov.argtypes = [C.POINTER(_Problem), P, C.POINTER(_NewtonOpts), C.POINTER(_NewtonStats),
                                       P, I64, C.POINTER(I64)]
        L.oc_sym_givens.argtypes = [D, D, P, P, P]
        L.oc_jacobian_diag.argtypes = [C.POINTER(_Problem), P, P, C.c_int]
        L.oc_ilu0_factor.argtypes = [C.POINTER(_Problem), P, P]
        L.oc_ilu0_solve.argtypes = [C.POINTER(_Problem), P, P, P]
        L.oc_set_threads.argtypes = [C.c_int]
        L.oc_set_chunk.argtypes = [C.c_int64]
        L.oc_set_devred.argtypes = [C.c_int, C.c_int, C.c_int]
        L.oc_set_devred_ranks.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int]
        L.oc_set_devred_user.argtypes = [C.c_int]
        L.oc_dr_tile_parts3d.argtypes = [I64, I64, I64, C.c_int, P, P, P]
        L.oc_dr_tile_parts3d.restype = I64
        L.oc_get_devred.restype = C.c_int
        L.oc_dr_ri.argtypes = [P, I64]
        L.oc_dr_ri.restype = D
        L.oc_dr_poll1.argtypes = [P, I64]
        L.oc_dr_poll1.restype = D
        L.oc_dr_chunk_parts.argtypes = [I64, P, P, I64, P]
        L.oc_dr_sweep_parts.argtypes = [I64, P, P, I64, P]
        L.oc_dr_tile_parts2d.argtypes = [I64, I64, P, P, P]
        L.oc_dr_tile_parts2d.restype = I64
        L.oc_get_threads.restype = C.c_int
        for name in ("oc_axpy",):
            getattr(L, name).argtypes = [I64, D, P, P]
        L.oc_axpby.argtypes = [I64, D, P, D, P]
        L.oc_exp.argtypes = [I64, P, P]
        L.oc_exp_slow.argtypes = [I64, P, P]
        L.oc_exp_dd.argtypes = [I64, P, P, P, C.POINTER(C.c_int32)]
        L.oc_exp_dd.restype = I64
        _lib = L
    return _lib


LIBM_PATH = os.path.join(HERE, "_build", "libnkoracle_libm.so")
_libm = None


def libm_variant():
    """The oracle built with the platform libm's exp (glibc) instead of nk_exp.h -- a cross-check of the
    shared correctly rounded exp (tests/test_oracle.py); residual / exact JVP / FD operator only."""
    global _libm
    if _libm is None:
        lib()  # (builds both)
        if not os.path.exists(LIBM_PATH):
            build()
        L = C.CDLL(LIBM_PATH)
        D, P = C.c_double, C.POINTER(C.c_double)
        L.oc_residual.argtypes = [C.POINTER(_Problem), P, P]
        L.oc_jv_exact.argtypes = [C.POINTER(_Problem), P, P, P]
        L.oc_jv_fd.argtypes = [C.POINTER(_Problem), P, P, P, P, D]
        L.oc_exp.argtypes = [C.c_int64, P, P]
        _libm = L
    return _libm


def _p(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_double))


@dataclass
class Problem:
    """Grid problem: kind + interior dims (x fastest) + parameters (see nk_oracle.c)."""
    kind: int
    nx: int
    ny: int = 1
    nz: int = 1
    hx: float = 1.0
    hy: float = 1.0
    hz: float = 1.0
    lam: float = 0.0
    a: float = 0.0
    dt: float = 0.0
    un: np.ndarray | None = field(default=None, repr=False)
    bc: int = BC_ZERO
    alpha: float = 0.5  # G_Midpoint! α (implicit.jl:17)

    @property
    def n(self) -> int:
        return self.nx * self.ny * self.nz

    @property
    def shape(self):
        return {1: (self.nx,), 2: (self.ny, self.nx), 3: (self.nz, self.ny, self.nx)}[self.dim]

    @property
    def dim(self) -> int:
        if self.kind == BRATU1D:
            return 1
        return 3 if self.kind in (HEAT3D_EULER, HEAT3D_MIDPOINT, HEAT3D_TRAPEZOID) else 2

    def _c(self) -> _Problem:
        s = _Problem(self.kind, self.bc, self.nx, self.ny, self.nz, self.hx, self.hy, self.hz, self.lam, self.a,
                     self.dt, None, self.alpha)
        if self.un is not None:
            self._un_keep = np.ascontiguousarray(self.un, dtype=np.float64).reshape(-1)
            assert self._un_keep.size == self.n
            s.un = _p(self._un_keep)
        return s


# -- problem constructors (parameters of the reference examples / SURVEY.md §8d) -------------------
LAMBDA_BRATU = 3.51382  # examples/bratu.jl:41


def bratu1d(N: int, lam: float = LAMBDA_BRATU) -> Problem:
    dx = 1.0 / (N + 1)  # bratu.jl:42
    return Problem(BRATU1D, N, hx=dx, lam=lam)


def bratu2d(nx: int, ny: int | None = None, lam: float = LAMBDA_BRATU) -> Problem:
    ny = nx if ny is None else ny
    return Problem(BRATU2D, nx, ny, hx=1.0 / (nx + 1), hy=1.0 / (ny + 1), lam=lam)


def heat_dt_2d(hx, hy, a):
    return hx ** 2 * hy ** 2 / (2.0 * a * (hx ** 2 + hy ** 2))  # heat_2D.jl:72


def heat2d_euler(nx: int, ny: int | None = None, a: float = 0.01, dt: float | None = None, un=None,
                 scheme: str = "euler", bc: int = BC_ZERO, alpha: float = 0.5) -> Problem:
    """G!(res, u_n, Δt, diffusion!, du, u, (a, Δx, Δy, bc!), t) for G in implicit.jl:8-37."""
    ny = nx if ny is None else ny
    hx, hy = 1.0 / (nx + 1), 1.0 / (ny + 1)
    dt = heat_dt_2d(hx, hy, a) if dt is None else dt
    return Problem(HEAT_KINDS[scheme, 2], nx, ny, hx=hx, hy=hy, a=a, dt=dt, un=un, bc=bc, alpha=alpha)


def heat_dt_3d(hx, hy, hz, a):
    return 1.0 / (2.0 * a * (1.0 / hx ** 2 + 1.0 / hy ** 2 + 1.0 / hz ** 2))


def heat3d_euler(nx: int, ny=None, nz=None, a: float = 0.01, dt=None, un=None, scheme: str = "euler",
                 bc: int = BC_ZERO, alpha: float = 0.5) -> Problem:
    ny = nx if ny is None else ny
    nz = nx if nz is None else nz
    hx, hy, hz = 1.0 / (nx + 1), 1.0 / (ny + 1), 1.0 / (nz + 1)
    dt = heat_dt_3d(hx, hy, hz, a) if dt is None else dt
    return Problem(HEAT_KINDS[scheme, 3], nx, ny, nz, hx=hx, hy=hy, hz=hz, a=a, dt=dt, un=un, bc=bc, alpha=alpha)


def sin_ic(P: Problem) -> np.ndarray:
    """u0 = sin(pi x) [sin(pi y) [sin(pi z)]] on the interior nodes h, 2h, ... (bratu.jl:45-46)."""
    xs = [np.arange(1, m + 1) * h for m, h in ((P.nx, P.hx), (P.ny, P.hy), (P.nz, P.hz))][: P.dim]
    out = np.sin(np.pi * xs[0])
    if P.dim >= 2:
        out = np.sin(np.pi * xs[1])[:, None] * out[None, :]
    if P.dim == 3:
        out = np.sin(np.pi * xs[2])[:, None, None] * out[None, :, :]
    return np.ascontiguousarray(out, dtype=np.float64)


# -- kernels -------------------------------------------------------------------------------------
def residual(P: Problem, u: np.ndarray, libm: bool = False) -> np.ndarray:
    """F!(res, u, p) (libm: with the platform exp instead of the shared correctly rounded one)."""
    u = np.ascontiguousarray(u, dtype=np.float64)
    res = np.empty_like(u)
    cp = P._c()
    (libm_variant() if libm else lib()).oc_residual(C.byref(cp), _p(res), _p(u))
    return res


def jv_exact(P: Problem, u, v, libm: bool = False) -> np.ndarray:
    u = np.ascontiguousarray(u, dtype=np.float64)
    v = np.ascontiguousarray(v, dtype=np.float64)
    out = np.empty_like(u)
    cp = P._c()
    (libm_variant() if libm else lib()).oc_jv_exact(C.byref(cp), _p(out), _p(u), _p(v))
    return out


def jacobian_diag(P: Problem, u, reciprocal=False) -> np.ndarray:
    """diag(J(u)) -- the diagonal of collect(J) (src/Ariadne.jl:140-162); reciprocal: Jacobi's 1 ./ diag."""
    u = np.ascontiguousarray(u, dtype=np.float64)
    out = np.empty_like(u)
    cp = P._c()
    lib().oc_jacobian_diag(C.byref(cp), _p(out), _p(u), int(bool(reciprocal)))
    return out


def ilu0_factor(P: Problem, u) -> np.ndarray:
    """The pivots D~ of ILU(0) of J(u) (see nk_oracle.c oc_ilu0_factor)."""
    u = np.ascontiguousarray(u, dtype=np.float64)
    d = np.empty_like(u)
    cp = P._c()
    lib().oc_ilu0_factor(C.byref(cp), _p(u), _p(d))
    return d


def ilu0_solve(P: Problem, d, v) -> np.ndarray:
    d = np.ascontiguousarray(d, dtype=np.float64)
    v = np.ascontiguousarray(v, dtype=np.float64)
    z = np.empty_like(v)
    cp = P._c()
    lib().oc_ilu0_solve(C.byref(cp), _p(d), _p(z), _p(v))
    return z


def _precond(N):
    """N = None | ("diag", d) | ("ilu0", D~) | ("gmres", itmax) -> (_Precond or None, keep-alive).
    (ILU0 reads J's off-diagonals from the solve's own problem.)"""
    if N is None:
        return None, None
    kind, arg = N
    if kind in ("diag", "ilu0"):
        d = np.ascontiguousarray(arg, dtype=np.float64).reshape(-1)
        return _Precond(PRECOND_DIAG if kind == "diag" else PRECOND_ILU0, 0, _p(d), None), d
    if kind == "gmres":
        return _Precond(PRECOND_GMRES, int(arg), None, None), None
    raise ValueError(kind)


def fd_eps(unorm: float, vnorm: float) -> float:
    return lib().oc_fd_eps(unorm, vnorm)


def jv_fd(P: Problem, u, v, F0=None, eps: float | None = None, libm: bool = False) -> np.ndarray:
    u = np.ascontiguousarray(u, dtype=np.float64)
    v = np.ascontiguousarray(v, dtype=np.float64)
    F0 = residual(P, u, libm=libm) if F0 is None else np.ascontiguousarray(F0, dtype=np.float64)
    if eps is None:
        eps = fd_eps(norm(u), norm(v))
    out = np.empty_like(u)
    cp = P._c()
    (libm_variant() if libm else lib()).oc_jv_fd(C.byref(cp), _p(out), _p(u), _p(v), _p(F0), eps)
    return out


def dot(x, y) -> float:
    x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1)
    y = np.ascontiguousarray(y, dtype=np.float64).reshape(-1)
    return lib().oc_dot(x.size, _p(x), _p(y))


def norm(x) -> float:
    x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1)
    return lib().oc_norm(x.size, _p(x))


def sym_givens(a: float, b: float):
    c, s, r = C.c_double(), C.c_double(), C.c_double()
    lib().oc_sym_givens(a, b, C.byref(c), C.byref(s), C.byref(r))
    return c.value, s.value, r.value


def ew_forcing(eta, tol, n_res, n_res_prior, eta_max=0.999, gamma=0.9):
    return lib().oc_ew_forcing(eta_max, gamma, eta, tol, n_res, n_res_prior)


def set_chunk(c: int):
    """Reduction chunk of the oracle's dot / norm (default 8192): another summation order."""
    lib().oc_set_chunk(int(c))


def set_devred(on: bool, cus: int = 256, rl: int = 39, ranks=(1, 1, 1), resident: bool = True, user: bool = False):
    """Sum the 2D / 3D GMRES reductions in exactly the device's order (nk_oracle.c OC_DEVRED): the kernels'
    trees -- wave butterflies, block sums, reduce_input, the chunked streaming kernels, k_st2d's / k_st3l's
    tiles and the resident sweep's slot partition over `cus` blocks (the GPU's CU count) -- so that
    restarted FD-GMRES histories compare bit for bit at any length.  ranks = (px, py, pz): the decomposition
    (3D blocks / z-slabs; 2D slabs are (1, R, 1)), each rank's tree over its own block and the ranks' sums
    added in rank order, as the peer mailbox adds them; resident: whether the ranks' MGS sweeps ran resident
    (ranks sharing one GPU run the per-pass chain); user: the device evaluated the residual through a user
    callback (NK_USER*), whose reductions are k_user_epi's scalar chunks instead of the stencil's tiles."""
    lib().oc_set_devred(int(bool(on)), int(cus), int(rl))
    lib().oc_set_devred_ranks(*(int(t) for t in ranks), int(bool(resident)))
    lib().oc_set_devred_user(int(bool(user)))  # user: the device ran the problem as a user residual (k_user_epi)


def get_devred() -> bool:
    return bool(lib().oc_get_devred())


def dr_trees(n: int, x, y=None, *, G: int = 256, nx: int = 0, ny: int = 0):
    """The device-order trees as separate pieces (CPU tests pin them against a Python restatement):
    chunk / sweep partials over G blocks, their reduce_input / polling-wave sums, k_st2d tile partials."""
    x = np.ascontiguousarray(x, dtype=np.float64).ravel()
    y = x if y is None else np.ascontiguousarray(y, dtype=np.float64).ravel()
    chunk = np.zeros(G)
    sweep = np.zeros(G)
    lib().oc_dr_chunk_parts(n, _p(x), _p(y), G, _p(chunk))
    lib().oc_dr_sweep_parts(n, _p(x), _p(y), G, _p(sweep))
    out = dict(chunk=chunk, sweep=sweep, ri_chunk=lib().oc_dr_ri(_p(chunk), G), poll1=lib().oc_dr_poll1(_p(sweep), G))
    if nx:
        nt = lib().oc_dr_tile_parts2d(nx, ny, _p(x), _p(y), None)
        tiles = np.zeros(nt)
        lib().oc_dr_tile_parts2d(nx, ny, _p(x), _p(y), _p(tiles))
        out.update(tiles=tiles, ri_tiles=lib().oc_dr_ri(_p(tiles), nt))
    return out


def set_threads(t: int):
    lib().oc_set_threads(int(t))


def get_threads() -> int:
    return lib().oc_get_threads()


def krylov_solve(P: Problem, u, b, *, algo="gmres", jv="exact", F0=None, memory=20, restart=False,
                 reorthogonalization=False, itmax=0, atol=SQRT_EPS, rtol=SQRT_EPS, history=True, N=None, M=None):
    """One Krylov.jl-style solve of J(u) x = b; returns (x, stats dict, residual-norm history).
    algo: gmres | fgmres | cg; N: right preconditioner ("diag", d), ("ilu0", D~) or ("gmres", itmax);
    M: left preconditioner, the same forms (cg: M is the SPD preconditioner)."""
    u = np.ascontiguousarray(u, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    if jv == "fd" and F0 is None:
        F0 = residual(P, u)
    F0 = np.ascontiguousarray(F0 if F0 is not None else u, dtype=np.float64)
    x = np.empty_like(u)
    Np, _keep = _precond(N)
    Mp, _keepm = _precond(M)
    o = _KrylovOpts(memory, int(restart), int(reorthogonalization), itmax, atol, rtol, int(algo == "fgmres"),
                    C.pointer(Np) if Np is not None else None, C.pointer(Mp) if Mp is not None else None)
    st = _KrylovStats()
    cap = (itmax if itmax else 2 * P.n) + 16 if history else 0
    cap = min(cap, 1 << 22)
    hist = np.zeros(max(cap, 1))
    hl = C.c_int64(0)
    cp = P._c()
    lib().oc_krylov_solve(C.byref(cp), JV_FD if jv == "fd" else JV_EXACT, _ALGO[algo],
                          _p(u), _p(F0), _p(b), _p(x), C.byref(o), C.byref(st), _p(hist), cap, C.byref(hl))
    stats = dict(niter=st.niter, solved=bool(st.solved), inconsistent=bool(st.inconsistent),
                 breakdown=bool(st.breakdown), status=st.status, n_matvec=st.n_matvec)
    return x, stats, hist[: min(hl.value, cap)].copy()


def newton_krylov(P: Problem, u0, *, tol_rel=1e-6, tol_abs=1e-12, max_niter=50, forcing="ew", eta=0.1,
                  eta_max=0.999, gamma=0.9, algo="gmres", jv="exact", memory=20, restart=False,
                  reorthogonalization=False, itmax=0, atol=SQRT_EPS, rtol=None, N=None, M=None):
    """Ariadne newton_krylov! restated (src/Ariadne.jl:288-372). rtol given => krylov_kwargs rtol wins.
    N: a factory called per Newton step -- "jacobi" (1 ./ diag(J(u))) or ("gmres", itmax), the
    GmresPreconditioner of examples/bratu.jl:139-157; M: the same factories for the left preconditioner
    (Ariadne.jl:327-329)."""
    u = np.array(u0, dtype=np.float64, order="C", copy=True)
    fk = {"none": FORCING_NONE, None: FORCING_NONE, "fixed": FORCING_FIXED, "ew": FORCING_EW}[forcing]
    ko = _KrylovOpts(memory, int(restart), int(reorthogonalization), itmax, atol, 0.0 if rtol is None else rtol)
    def factory(F):
        if F is None:
            return PRECOND_NONE, 0
        if F == "jacobi":
            return PRECOND_JACOBI, 0
        if F == "ilu":
            return PRECOND_ILU, 0
        return PRECOND_GMRES, int(F[1])
    pk, pit = factory(N)
    mk, mit = factory(M)
    o = _NewtonOpts(tol_rel, tol_abs, max_niter, fk, eta, eta_max, gamma,
                    _ALGO[algo], JV_FD if jv == "fd" else JV_EXACT, ko,
                    0 if rtol is None else 1, pk, pit, mk, mit)
    st = _NewtonStats()
    cap = max_niter + 4
    hist = np.zeros(cap)
    inner = np.zeros(cap, dtype=np.int64)
    cp = P._c()
    lib().oc_newton_krylov(C.byref(cp), _p(u), C.byref(o), C.byref(st), _p(hist), cap,
                           inner.ctypes.data_as(C.POINTER(C.c_int64)))
    k = st.outer_iterations
    stats = dict(outer_iterations=st.outer_iterations, inner_iterations=st.inner_iterations, n_res=st.n_res,
                 solved=bool(st.solved), n_matvec=st.n_matvec, n_residual=st.n_residual, tol=st.tol,
                 n_res_history=hist[: k + 1].copy(), inner_history=inner[:k].copy())
    return u, stats


def _blas1(name, *args):
    getattr(lib(), name)(*args)


def axpy(s, x, y):
    """y + s x with fma (Krylov kaxpy! on dense vectors); returns a new array."""
    x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1)
    y = np.array(y, dtype=np.float64).reshape(-1)
    lib().oc_axpy(x.size, float(s), _p(x), _p(y))
    return y


def axpby(s, x, t, y):
    """s x + t y as fma(t, y, s*x) (Krylov kaxpby!); returns a new array."""
    x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1)
    y = np.array(y, dtype=np.float64).reshape(-1)
    lib().oc_axpby(x.size, float(s), _p(x), float(t), _p(y))
    return y


# ----------------------------------------------------------------------------- the shared exp
def exp(x) -> np.ndarray:
    """nk_exp (csrc/nk_exp.h): the correctly rounded exp every Bratu evaluation uses, elementwise."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    lib().oc_exp(x.size, _p(x), _p(y))
    return y


def exp_slow(x) -> np.ndarray:
    """nk_exp's exact fixed-point phase alone (valid for 2^-54 < |x| < 746)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    lib().oc_exp_slow(x.size, _p(x), _p(y))
    return y


def exp_dd(x):
    """nk_exp's fast phase alone: (zh, zl, m) with exp(x) ~ (zh + zl) 2^m, and how many inputs its Ziv
    test would hand to the exact phase."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    zh, zl = np.empty_like(x), np.empty_like(x)
    m = np.empty(x.shape, dtype=np.int32)
    slow = lib().oc_exp_dd(x.size, _p(x), _p(zh), _p(zl), m.ctypes.data_as(C.POINTER(C.c_int32)))
    return zh, zl, m, int(slow)
