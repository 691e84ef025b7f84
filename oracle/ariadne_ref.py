"""Pure-Python/numpy restatement of Ariadne's JFNK driver for SMALL generic problems.

TEST INFRASTRUCTURE ONLY (see oracle/oracle.py header): only tests/ may import it.

Why a second restatement: the C oracle (nk_oracle.c) is specialised to grid stencils; the
reference's own tests (test/runtests.jl) exercise a generic 2x2 residual written as a
Julia function and differentiated by Enzyme.  Here the residual is any Python callable
``F_(res, x, p)`` and the JVP is forward-mode AD with dual numbers -- the same semantics as
``autodiff(Forward, F!, Duplicated(res, out), Duplicated(u, v), p)`` (src/Ariadne.jl:48-57),
and ``collect(J)`` (:140-162).  The Newton loop follows src/Ariadne.jl:288-372 line by line;
GMRES/CG follow Krylov.jl 0.10 (third-party, parity unpinned).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

EPS = float(np.finfo(np.float64).eps)
SQRT_EPS = math.sqrt(EPS)


# ----------------------------------------------------------------------------- dual numbers
class Dual:
    """Forward-mode dual number: value + eps * tangent."""

    __slots__ = ("v", "d")

    def __init__(self, v, d=0.0):
        self.v = float(v)
        self.d = float(d)

    @staticmethod
    def lift(x):
        return x if isinstance(x, Dual) else Dual(x, 0.0)

    def __add__(self, o):
        o = Dual.lift(o)
        return Dual(self.v + o.v, self.d + o.d)

    __radd__ = __add__

    def __sub__(self, o):
        o = Dual.lift(o)
        return Dual(self.v - o.v, self.d - o.d)

    def __rsub__(self, o):
        return Dual.lift(o) - self

    def __mul__(self, o):
        o = Dual.lift(o)
        return Dual(self.v * o.v, self.d * o.v + self.v * o.d)

    __rmul__ = __mul__

    def __truediv__(self, o):
        o = Dual.lift(o)
        if o.d == 0.0:  # Enzyme's forward FDiv: dx/c + (-(x dc)/c²) with dc = 0 is dx/c exactly
            return Dual(self.v / o.v, self.d / o.v)
        return Dual(self.v / o.v, (self.d * o.v - self.v * o.d) / (o.v * o.v))

    def __rtruediv__(self, o):
        return Dual.lift(o) / self

    def __neg__(self):
        return Dual(-self.v, -self.d)

    def __pow__(self, k):
        if isinstance(k, int) and k == 2:  # Julia literal_pow: x^2 == x*x
            return self * self
        k = float(k)
        return Dual(self.v ** k, k * self.v ** (k - 1) * self.d)


def dexp(x):
    if isinstance(x, Dual):
        e = math.exp(x.v)
        return Dual(e, e * x.d)
    return math.exp(x)


def _dual_array(vals, tans):
    out = np.empty(len(vals), dtype=object)
    for i, (a, b) in enumerate(zip(vals, tans)):
        out[i] = Dual(a, b)
    return out


def jvp(F_, u, v, p=None):
    """(F(u), J(u) v) by forward mode; F_ writes into res like F!(res, u, p)."""
    u = np.asarray(u, dtype=np.float64)
    x = _dual_array(u, np.asarray(v, dtype=np.float64))
    res = np.empty(u.size, dtype=object)
    res[:] = [Dual(0.0) for _ in range(u.size)]
    F_(res, x, p)
    val = np.array([Dual.lift(r).v for r in res])
    tan = np.array([Dual.lift(r).d for r in res])
    return val, tan


def collect(F_, u, p=None):
    """collect(J): n unit-vector matvecs (src/Ariadne.jl:140-162), dense here."""
    n = len(u)
    J = np.zeros((n, n))
    for j in range(n):
        e = np.zeros(n)
        e[j] = 1.0
        J[:, j] = jvp(F_, u, e, p)[1]
    return J


def vjp(F_, u, w, p=None):
    """J(u)^T w (the reverse-mode transpose mul!, src/Ariadne.jl:93-107), via the dense Jacobian."""
    return collect(F_, u, p).T @ np.asarray(w, dtype=np.float64)


# ----------------------------------------------------------------------------- Krylov.jl restatements
def sym_givens(a, b):
    if b == 0.0:
        c = 1.0 if a == 0.0 else math.copysign(1.0, a)
        return c, 0.0, abs(a)
    if a == 0.0:
        return 0.0, math.copysign(1.0, b), abs(b)
    if abs(b) > abs(a):
        t = a / b
        s = math.copysign(1.0, b) / math.sqrt(1.0 + t * t)
        c = s * t
        return c, s, b / s
    t = b / a
    c = math.copysign(1.0, a) / math.sqrt(1.0 + t * t)
    s = c * t
    return c, s, a / c


@dataclass
class KrylovStats:
    niter: int = 0
    solved: bool = False
    inconsistent: bool = False
    status: str = "unknown"


def gmres(A, b, *, memory=20, restart=False, reorthogonalization=False, atol=SQRT_EPS, rtol=SQRT_EPS, itmax=0,
          dot=None, n=None, M=None):
    """Krylov.jl gmres! with N = I. A: callable v -> A v; M: the left
    preconditioner as a callable v -> M v (ldiv = false; None = I): r0 = M w, q = M A V_k.

    `dot` (default numpy) lets a caller supply a distributed inner product (all-reduced over
    ranks) and `n` the global length -- the multi-rank protocol test uses both."""
    dot = dot or (lambda x, y: float(np.dot(x, y)))
    n = b.size if n is None else n  # global length (itmax = 2n); arrays are this rank's b.size
    x = np.zeros(b.size)
    xr = np.zeros(b.size) if restart else x
    Mf = M or (lambda v: v)
    w = Mf(b.copy())  # r0 = M (b - A 0)
    beta = math.sqrt(dot(w, w))
    rNorm = beta
    hist = [rNorm]
    eps_ = atol + rtol * rNorm
    st = KrylovStats()
    if beta == 0.0:
        st.solved = True
        st.status = "x = 0 is a zero-residual solution"
        return x, st, hist
    npass, it = 0, 0
    itmax = 2 * n if itmax == 0 else itmax
    inner_itmax = itmax
    btol = EPS ** 0.75
    breakdown = inconsistent = False
    solved = rNorm <= eps_
    tired = it >= itmax
    nmv = 0
    while not (solved or tired or breakdown):
        V, R, c, s, z = [], [], [], [], [0.0]
        if restart:
            xr[:] = 0.0
            if npass >= 1:
                w = Mf(b - A(x))
                nmv += 1
        beta = math.sqrt(dot(w, w))
        z[0] = beta
        V.append(w / rNorm)  # kdivcopy!(n, V[1], r0, rNorm): after a restart, the previous cycle's estimate
        npass += 1
        k = 0
        inner_tired = False
        while not (solved or inner_tired or breakdown):
            k += 1
            w = Mf(A(V[k - 1]))
            nmv += 1
            col = []
            for i in range(k):
                h = dot(V[i], w)
                col.append(h)
                w = w - h * V[i]
            if reorthogonalization:
                for i in range(k):
                    h = dot(V[i], w)
                    col[i] += h
                    w = w - h * V[i]
            Hbis = math.sqrt(dot(w, w))
            for i in range(k - 1):
                rtmp = c[i] * col[i] + s[i] * col[i + 1]
                col[i + 1] = s[i] * col[i] - c[i] * col[i + 1]
                col[i] = rtmp
            ck, sk, col[k - 1] = sym_givens(col[k - 1], Hbis)
            c.append(ck)
            s.append(sk)
            R.append(col)
            zeta = sk * z[k - 1]
            z[k - 1] = ck * z[k - 1]
            rNorm = abs(zeta)
            hist.append(rNorm)
            solved = rNorm <= eps_ or (rNorm + 1.0 <= 1.0)
            breakdown = Hbis <= btol
            inner_tired = k >= min(memory, inner_itmax) if restart else k >= inner_itmax
            if not (solved or inner_tired or breakdown):
                V.append(w / Hbis)
                z.append(zeta)
        y = list(z[:k])
        for i in range(k - 1, -1, -1):
            for j in range(k - 1, i, -1):
                y[i] = y[i] - R[j][i] * y[j]
            if abs(R[i][i]) <= btol:
                y[i] = 0.0
                inconsistent = True
            else:
                y[i] = y[i] / R[i][i]
        for i in range(k):
            xr += y[i] * V[i]
        if restart:
            x += xr
        it += k
        inner_itmax = itmax - it
        tired = it >= itmax
    st.niter, st.solved, st.inconsistent = it, solved, inconsistent
    st.status = "solved" if solved else ("tired" if tired else "breakdown")
    return x, st, hist


def cg(A, b, *, atol=SQRT_EPS, rtol=SQRT_EPS, itmax=0, M=None):
    """Krylov.jl cg! with radius = 0, linesearch = false; M: the (SPD) preconditioner as a callable
    (None = I): z = M r, gamma = <r, z>, p = z + beta p."""
    Mf = M or (lambda v: v)
    n = b.size
    x = np.zeros(n)
    r = b.copy()
    z = Mf(r)
    p = z.copy()
    gamma = float(np.dot(r, z))
    rNorm = math.sqrt(gamma)
    hist = [rNorm]
    st = KrylovStats()
    if gamma == 0.0:
        st.solved = True
        return x, st, hist
    itmax = 2 * n if itmax == 0 else itmax
    pN2 = gamma
    eps_ = atol + rtol * rNorm
    it, solved, tired, zc = 0, rNorm <= eps_, False, False
    while not (solved or tired or zc):
        Ap = A(p)
        pAp = float(np.dot(p, Ap))
        if pAp <= EPS * pN2 and abs(pAp) <= EPS * pN2:
            zc = True
            st.inconsistent = True
            continue
        alpha = gamma / pAp
        x += alpha * p
        r -= alpha * Ap
        z = Mf(r)
        gn = float(np.dot(r, z))
        rNorm = math.sqrt(gn)
        hist.append(rNorm)
        solved = rNorm <= eps_ or rNorm + 1.0 <= 1.0
        if not solved:
            beta = gn / gamma
            pN2 = gn + beta * beta * pN2
            gamma = gn
            p = z + beta * p
        it += 1
        tired = it >= itmax
    st.niter, st.solved = it, solved
    return x, st, hist


# ----------------------------------------------------------------------------- Ariadne
@dataclass(frozen=True)
class Fixed:
    """Fixed(η = 0.1) -- src/Ariadne.jl:185-192."""
    eta: float = 0.1

    def __call__(self, *args):
        return self.eta

    def initial(self):
        return self.eta


@dataclass(frozen=True)
class EisenstatWalker:
    """EisenstatWalker(η_max = 0.999, γ = 0.9) -- src/Ariadne.jl:197-217."""
    eta_max: float = 0.999
    gamma: float = 0.9

    def __call__(self, eta, tol, n_res, n_res_prior):
        eta_res = self.gamma * n_res ** 2 / n_res_prior ** 2
        # `γ η^2 <= 1 // 10` is an exact rational comparison: for a double that is `< 0.1`
        if self.gamma * eta ** 2 < 0.1:
            eta_safe = min(self.eta_max, eta_res)
        else:
            eta_safe = min(self.eta_max, max(eta_res, self.gamma * eta ** 2))
        return min(self.eta_max, max(eta_safe, 0.5 * tol / n_res))

    def initial(self):
        return self.eta_max


def newton_krylov_(F_, u, p=None, res=None, *, tol_rel=1e-6, tol_abs=1e-12, max_niter=50,
                   forcing=EisenstatWalker(), algo="gmres", krylov_kwargs=None, callback=None, memory=20):
    """src/Ariadne.jl:288-372 restated for generic callables (JVP by dual numbers)."""
    u = np.array(u, dtype=np.float64)
    res = np.zeros_like(u) if res is None else res
    krylov_kwargs = dict(krylov_kwargs or {})
    F_(res, u, p)
    n_res = float(np.linalg.norm(res))
    callback and callback(u, res, n_res)
    tol = tol_rel * n_res + tol_abs
    eta = forcing.initial() if forcing is not None else None
    outer = inner = 0
    while n_res > tol and outer <= max_niter:
        kw = dict(krylov_kwargs)
        if forcing is not None:
            kw = {"rtol": eta, **kw}
        A = lambda v, _u=u.copy(): jvp(F_, _u, v, p)[1]
        if algo == "cg":
            d, kst, _ = cg(A, res.copy(), **kw)
        else:
            d, kst, _ = gmres(A, res.copy(), memory=memory, **kw)
        u -= d
        n_prior = n_res
        F_(res, u, p)
        n_res = float(np.linalg.norm(res))
        callback and callback(u, res, n_res)
        if math.isinf(n_res) or math.isnan(n_res):
            break
        if forcing is not None:
            eta = forcing(eta, tol, n_res, n_prior)
        outer += 1
        inner += kst.niter
    return u, dict(solved=n_res <= tol, outer_iterations=outer, inner_iterations=inner, n_res=n_res)


def newton_krylov(F, u0, p=None, **kw):
    """Out-of-place form (src/Ariadne.jl:245-248)."""
    def F_(res, u, p):
        res[:] = F(u, p)
    return newton_krylov_(F_, u0, p, **kw)


# ----------------------------------------------------------------------------- heat examples on halo arrays
# A literal restatement of examples/heat_2D.jl (bc_periodic!, bc_zero!, diffusion!) and
# examples/implicit.jl (G_Euler!, G_Midpoint!, G_Trapezoid!) on (N+2) x (M+2) halo arrays indexed
# [i, j] like the reference's OffsetArray (i = x, the column-major fast index; 0 and N+1 are ghosts).
# Arrays may hold Dual numbers: evaluating G! on u = Dual(u, v) gives F(u) and the forward-mode
# tangent J(u) v, independently of the C oracle's hand-derived tangents.
def bc_periodic_h(u):
    """heat_2D.jl:15-26 (note: N is reused for the second dimension -- square grids)."""
    N, M = u.shape
    N, M = N - 2, M - 2
    u[0, :] = u[N, :]
    u[N + 1, :] = u[1, :]
    u[:, 0] = u[:, N]
    u[:, N + 1] = u[:, 1]


def bc_zero_h(u):
    """heat_2D.jl:28-38."""
    N, M = u.shape
    N, M = N - 2, M - 2
    u[0, :] = 0.0
    u[N + 1, :] = 0.0
    u[:, 0] = 0.0
    u[:, N + 1] = 0.0


def diffusion_h(du, u, p, _t):
    """heat_2D.jl:45-62: bc!(u), then the 5-point Laplacian, i outer / j inner."""
    a, dx, dy, bc = p
    N, M = u.shape
    N, M = N - 2, M - 2
    bc(u)
    for i in range(1, N + 1):
        for j in range(1, M + 1):
            du[i, j] = a * ((u[i + 1, j] - 2 * u[i, j] + u[i - 1, j]) / (dx * dx)
                            + (u[i, j + 1] - 2 * u[i, j] + u[i, j - 1]) / (dy * dy))


def _interior(x):
    return x[1:-1, 1:-1]


def G_Euler_h(res, un, dt, f, du, u, p, t):
    """implicit.jl:8-13."""
    f(du, u, p, t)
    _interior(res)[...] = _interior(un) + dt * _interior(du) - _interior(u)


def G_Midpoint_h(res, un, dt, f, du, u, p, t, alpha=0.5):
    """implicit.jl:17-25: res is the temporary for α uₙ + (1 - α) u (interior broadcast)."""
    uu = res
    _interior(uu)[...] = alpha * _interior(un) + (1 - alpha) * _interior(u)
    f(du, uu, p, t + alpha * dt)
    _interior(res)[...] = _interior(un) + dt * _interior(du) - _interior(u)


def G_Trapezoid_h(res, un, dt, f, du, u, p, t):
    """implicit.jl:29-37: res is the temporary for du(uₙ)."""
    dun = res
    f(dun, un, p, t)
    f(du, u, p, t + dt)
    _interior(res)[...] = _interior(un) + (dt / 2) * (_interior(dun) + _interior(du)) - _interior(u)


def heat_halo_jvp(G, un, u, v, a, dx, dy, dt, bc, **kw):
    """(G(u), J(u) v) of G!(res, uₙ, Δt, diffusion!, du, u, (a, Δx, Δy, bc!), t) on interior arrays
    shaped (M, N) (row-major, x fastest: the oracle layout); returns the same layout."""
    M, N = u.shape
    H = np.empty((N + 2, M + 2), dtype=object)
    for idx in np.ndindex(H.shape):
        H[idx] = Dual(0.0)
    Un = H.copy()
    for idx in np.ndindex(H.shape):
        Un[idx] = Dual(0.0)
    for j in range(M):
        for i in range(N):
            H[i + 1, j + 1] = Dual(u[j, i], v[j, i])
            Un[i + 1, j + 1] = Dual(un[j, i], 0.0)
    res = np.empty_like(H)
    du = np.empty_like(H)
    for idx in np.ndindex(H.shape):
        res[idx] = Dual(0.0)
        du[idx] = Dual(0.0)
    G(res, Un, dt, diffusion_h, du, H, (a, dx, dy, bc), 0.0, **kw)
    val = np.array([[Dual.lift(res[i + 1, j + 1]).v for i in range(N)] for j in range(M)])
    tan = np.array([[Dual.lift(res[i + 1, j + 1]).d for i in range(N)] for j in range(M)])
    return val, tan
