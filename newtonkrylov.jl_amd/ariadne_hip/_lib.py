"""ctypes binding of libnkhip.so (include/nkhip.h).

The product path has no CPU fallback: if the HIP library is missing or no GPU is visible,
every compute entry point raises.  (Only loading the library and reading its symbol table
works without a GPU -- that is what the CPU test-suite checks.)
"""
from __future__ import annotations

import ctypes as C
import os
import sys

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRODUCT_LIB = os.path.join(PKG_DIR, "lib", "libnkhip.so")
# the kernel-variant bench build of the same sources (tuning knobs from the environment, nkb_* hooks);
# NK_KBENCH_LIB=1 loads it instead -- tools/ and the variant-equivalence tests only
KBENCH_LIB = os.path.join(PKG_DIR, "lib", "libnkhip_kbench.so")
LIB_PATH = KBENCH_LIB if os.environ.get("NK_KBENCH_LIB") == "1" else PRODUCT_LIB
# A/B tools only: a product build with extra defines (`make variant TAG=...` -> lib/libnkhip_v_TAG.so)
if os.environ.get("NK_LIB_VARIANT"):
    LIB_PATH = os.path.join(PKG_DIR, "lib", f"libnkhip_v_{os.environ['NK_LIB_VARIANT']}.so")
HEADER = os.path.join(os.path.dirname(PKG_DIR), "include", "nkhip.h")

NK_OK = 0
NK_E_HIP, NK_E_ARG, NK_E_NOMEM, NK_E_RCCL, NK_E_STATE, NK_E_USER = -1, -2, -3, -4, -5, -6
NK_BRATU1D, NK_BRATU2D, NK_HEAT2D_EULER, NK_HEAT3D_EULER = 1, 2, 3, 4
NK_HEAT2D_MIDPOINT, NK_HEAT3D_MIDPOINT, NK_HEAT2D_TRAPEZOID, NK_HEAT3D_TRAPEZOID = 5, 6, 7, 8
NK_USER1D, NK_USER2D, NK_USER3D = 16, 17, 18
NK_BC_ZERO, NK_BC_PERIODIC = 0, 1
NK_JV_EXACT, NK_JV_FD = 0, 1
NK_ALGO_GMRES, NK_ALGO_CG, NK_ALGO_FGMRES = 0, 1, 2
NK_PRECOND_NONE, NK_PRECOND_DIAG, NK_PRECOND_USER, NK_PRECOND_GMRES, NK_PRECOND_ILU0 = 0, 1, 2, 3, 4

_ERRORS = {-1: "HIP error", -2: "invalid argument", -3: "out of device memory", -4: "RCCL error", -5: "bad state", -6: "user callback failed"}


class NKError(RuntimeError):
    pass


class nk_problem(C.Structure):
    _fields_ = [("kind", C.c_int32), ("bc", C.c_int32),
                ("nx", C.c_int64), ("ny", C.c_int64), ("nz", C.c_int64),
                ("hx", C.c_double), ("hy", C.c_double), ("hz", C.c_double),
                ("lam", C.c_double), ("a", C.c_double), ("dt", C.c_double),
                ("un", C.c_void_p), ("user", C.c_void_p), ("alpha", C.c_double)]


# nk_user_ops: int F(void* data, nk_ctx*, double* res, const double* u); int J(data, ctx, out, u, v)
NK_USER_RESIDUAL = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p)
NK_USER_TANGENT = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p)


NK_USER_PRECOND = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p)


class nk_precond(C.Structure):
    _fields_ = [("kind", C.c_int32), ("diag", C.c_void_p), ("apply", NK_USER_PRECOND), ("data", C.c_void_p),
                ("inner", C.c_void_p), ("itmax", C.c_int32)]


class nk_user_ops(C.Structure):
    _fields_ = [("F", NK_USER_RESIDUAL), ("J", NK_USER_TANGENT), ("JT", NK_USER_TANGENT), ("data", C.c_void_p)]


class nk_krylov_opts(C.Structure):
    _fields_ = [("restart", C.c_int32), ("reorthogonalization", C.c_int32), ("itmax", C.c_int32),
                ("jv_mode", C.c_int32), ("atol", C.c_double), ("rtol", C.c_double), ("b_norm", C.c_double),
                ("u_norm", C.c_double), ("u_update", C.c_void_p), ("N", C.c_void_p),
                ("M", C.c_void_p), ("f0_is_residual", C.c_int32)]


class nk_krylov_stats(C.Structure):
    _fields_ = [("niter", C.c_int64), ("solved", C.c_int32), ("inconsistent", C.c_int32),
                ("breakdown", C.c_int32), ("status", C.c_int32), ("n_matvec", C.c_int64), ("u_norm", C.c_double)]


NK_FORCING_NONE, NK_FORCING_FIXED, NK_FORCING_EW = 0, 1, 2


class nk_newton_opts(C.Structure):
    _fields_ = [("tol_rel", C.c_double), ("tol_abs", C.c_double), ("max_niter", C.c_int32), ("forcing", C.c_int32),
                ("eta", C.c_double), ("eta_max", C.c_double), ("gamma", C.c_double), ("algo", C.c_int32),
                ("memory", C.c_int32), ("krylov", nk_krylov_opts), ("rtol_user", C.c_int32)]


class nk_newton_stats(C.Structure):
    _fields_ = [("outer_iterations", C.c_int64), ("inner_iterations", C.c_int64), ("n_res", C.c_double),
                ("tol", C.c_double), ("solved", C.c_int32), ("n_matvec", C.c_int64), ("n_residual", C.c_int64)]


class nk_path_info(C.Structure):
    _fields_ = [("rank", C.c_int32), ("nranks", C.c_int32), ("device", C.c_int32), ("ranks_on_device", C.c_int32),
                ("rccl", C.c_int32), ("mailbox", C.c_int32), ("resident_sweep", C.c_int32),
                ("resident_blocks", C.c_int32), ("halo_in_launch", C.c_int32), ("mailbox_error", C.c_int32),
                ("halo_cap", C.c_int64), ("pci_bus_id", C.c_char * 32), ("jv_halo_fused", C.c_int64),
                ("jv_halo_separate", C.c_int64), ("sweeps_resident", C.c_int64), ("mgs_passes", C.c_int64),
                ("jv_fd_f0r", C.c_int64), ("jv_fd_f0_read", C.c_int64), ("halo_waits", C.c_int64),
                ("reduce_waits", C.c_int64), ("halo_wait_us", C.c_double), ("reduce_wait_us", C.c_double)]


class nk_prof_entry(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("launches", C.c_int64), ("timed", C.c_int64), ("total_ms", C.c_double),
                ("bytes", C.c_double), ("bytes_all", C.c_double), ("dram_bytes_all", C.c_double),
                ("kernel", C.c_char * 64)]


# name -> (restype, argtypes); mirrors include/nkhip.h one to one
_VP, _I32, _I64, _D, _PD = C.c_void_p, C.c_int32, C.c_int64, C.c_double, C.POINTER(C.c_double)
_PP = C.POINTER(nk_problem)
SIGNATURES = {
    "nk_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "nk_ctx_create": (C.c_int, [C.c_int, C.POINTER(_VP)]),
    "nk_ctx_destroy": (C.c_int, [_VP]),
    "nk_last_error": (C.c_char_p, [_VP]),
    "nk_sync": (C.c_int, [_VP]),
    "nk_ctx_stream": (_VP, [_VP]),
    "nk_vec_alloc": (C.c_int, [_VP, _PP, C.POINTER(_VP)]),
    "nk_vec_free": (C.c_int, [_VP, _VP]),
    "nk_memcpy_h2d": (C.c_int, [_VP, _VP, _VP, _I64]),
    "nk_memcpy_d2h": (C.c_int, [_VP, _VP, _VP, _I64]),
    "nk_residual": (C.c_int, [_VP, _PP, _VP, _VP]),
    "nk_residual_norm": (C.c_int, [_VP, _PP, _VP, _VP, _PD]),
    "nk_jv": (C.c_int, [_VP, _PP, _VP, _VP, _VP, _VP, _I32, _D]),
    "nk_jtv": (C.c_int, [_VP, _PP, _VP, _VP, _VP]),
    "nk_jv_batched": (C.c_int, [_VP, _PP, _I32, C.POINTER(_VP), _VP, C.POINTER(_VP), _VP, _I32, _D]),
    "nk_jtv_batched": (C.c_int, [_VP, _PP, _I32, C.POINTER(_VP), _VP, C.POINTER(_VP)]),
    "nk_jacobian_collect": (C.c_int, [_VP, _PP, _VP, _I32, C.POINTER(_I64), C.POINTER(_I64), _PD, _I64,
                                      C.POINTER(_I64)]),
    "nk_jacobian_diag": (C.c_int, [_VP, _PP, _VP, _VP, _I32]),
    "nk_ilu0_factor": (C.c_int, [_VP, _PP, _VP, _VP]),
    "nk_precond_apply": (C.c_int, [_VP, _PP, _VP, _VP, _VP, _I32, _VP, _VP]),
    "nk_dot": (C.c_int, [_VP, _I64, _VP, _VP, _PD]),
    "nk_mgs_step": (C.c_int, [_VP, _I64, C.POINTER(_VP), _I32, _VP, _I32, _PD]),
    "nk_norm": (C.c_int, [_VP, _I64, _VP, _PD]),
    "nk_scal": (C.c_int, [_VP, _I64, _D, _VP]),
    "nk_axpy": (C.c_int, [_VP, _I64, _D, _VP, _VP]),
    "nk_axpby": (C.c_int, [_VP, _I64, _D, _VP, _D, _VP]),
    "nk_copy": (C.c_int, [_VP, _I64, _VP, _VP]),
    "nk_axpy_norm": (C.c_int, [_VP, _I64, _D, _VP, _VP, _PD]),
    "nk_fill": (C.c_int, [_VP, _I64, _VP, _D]),
    "nk_divcopy": (C.c_int, [_VP, _I64, _VP, _VP, _D]),
    "nk_ref": (C.c_int, [_VP, _I64, _VP, _VP, _D, _D]),
    "nk_vexp": (C.c_int, [_VP, _I64, _VP, _VP]),
    "nk_workspace_create": (C.c_int, [_VP, _I32, _PP, _I32, C.POINTER(_VP)]),
    "nk_workspace_destroy": (C.c_int, [_VP]),
    "nk_workspace_x": (_VP, [_VP]),
    "nk_workspace_basis": (_VP, [_VP, _I32]),
    "nk_krylov_solve": (C.c_int, [_VP, _PP, _VP, _VP, _VP, C.POINTER(nk_krylov_opts), C.POINTER(nk_krylov_stats),
                                  _PD, _I64, C.POINTER(_I64)]),
    "nk_newton_defaults": (C.c_int, [C.POINTER(nk_newton_opts)]),
    "nk_newton_krylov": (C.c_int, [_VP, _PP, _VP, _VP, C.POINTER(nk_newton_opts), C.POINTER(nk_newton_stats),
                                   _PD, _I64, C.POINTER(_I64)]),
    "nk_dist_unique_id": (C.c_int, [C.c_char_p]),
    "nk_dist_init": (C.c_int, [_VP, _I32, _I32, C.c_char_p]),
    "nk_dist_allreduce_sum": (C.c_int, [_VP, _VP, _I64]),
    "nk_halo_exchange": (C.c_int, [_VP, _PP, _VP]),
    "nk_dist_mailbox_handle": (C.c_int, [_VP, C.c_char_p]),
    "nk_dist_mailbox_open": (C.c_int, [_VP, _I32, _I32, C.c_char_p]),
    "nk_dist_mailbox_active": (C.c_int, [_VP]),
    "nk_dist_path": (C.c_int, [_VP, C.POINTER(nk_path_info)]),
    "nk_dist_grid": (C.c_int, [_VP, _I32, _I32, _I32]),
    "nk_prof_enable": (C.c_int, [_VP, _I32]),
    "nk_prof_reset": (C.c_int, [_VP]),
    "nk_prof_read": (C.c_int, [_VP, C.POINTER(nk_prof_entry), _I32, C.POINTER(_I32)]),
}

_lib = None
TORCH_FIRST = False


def load():
    """Load libnkhip.so (built in-tree by __graft_entry__.build() / `make -C newtonkrylov.jl_amd`), or the
    kbench build when NK_KBENCH_LIB=1."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NKError(f"libnkhip.so not built ({LIB_PATH}); run `make -C newtonkrylov.jl_amd` -- "
                          "there is no CPU fallback")
        global TORCH_FIRST
        TORCH_FIRST = "torch" in sys.modules  # then libnkhip binds torch's HIP runtime (one runtime per process)
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        _lib = lib
    return _lib


_user_error = None


def set_user_error(e: BaseException):
    """A user-residual callback raised: remembered here, re-raised by the C call that ran it."""
    global _user_error
    _user_error = e


def require_torch_first():
    """torch interop needs ONE HIP runtime in the process: torch must be imported before libnkhip.so loads."""
    if not TORCH_FIRST:
        raise NKError("torch interop: import torch before ariadne_hip loads libnkhip.so, so that both use the "
                      "same HIP runtime (torch bundles its own)")


def check(rc: int, ctx=None, what: str = ""):
    global _user_error
    if rc != NK_OK:
        msg = ""
        if ctx is not None:
            m = load().nk_last_error(ctx)
            msg = m.decode() if m else ""
        cause, _user_error = _user_error, None
        if rc != -6:
            cause = None
        if cause is not None:
            msg += f" ({type(cause).__name__}: {cause})"
        raise NKError(f"{what}: {_ERRORS.get(rc, rc)} {msg}".strip()) from cause


def device_count() -> int:
    n = C.c_int(0)
    rc = load().nk_device_count(C.byref(n))
    return n.value if rc == NK_OK else 0
