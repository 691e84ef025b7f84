"""ariadne_hip -- MI355X-native JFNK inner loop behind Ariadne's API (host mirror, ctypes over libnkhip.so).

Reference: vchuravy/NewtonKrylov.jl (package Ariadne.jl), src/Ariadne.jl.  The Julia names map
1:1 with `!` -> trailing `_`:  newton_krylov! -> newton_krylov_, mul! -> mul_, kaxpy! -> kaxpy_.
"""
from ._lib import NKError, device_count, load
from .ariadne import (EisenstatWalker, Fixed, Forcing, JacobianOperator, Result, Stats, mul_, newton_krylov, newton_krylov_native, transpose, collect, TransposeOperator,
                      newton_krylov_)
from .device import Context, DeviceArray, Grid, default_context, set_default_context
from .distributed import block, dist_unique_id, init_distributed, slab
from .implicit import G_Euler_, G_Midpoint_, G_Trapezoid_, diffusion3d_, diffusion_, solve
from .krylov import (KrylovConstructor, exp_, kaxpby_, kaxpy_, kaxpy_norm_, kcopy_, kdivcopy_, kdot, kfill_, knorm, kref_, krylov_solve_,
                     krylov_workspace, kscal_, mgs_step_)
from .precond import (DiagonalPreconditioner, GmresPreconditioner, Ilu0Preconditioner, Preconditioner, UserPreconditioner,
                      gmres_preconditioner, ilu0, jacobi, jacobian_diag)
from .problems import (DeviceResidual, UserResidual, bc_periodic_, bc_zero_, bratu2d_, bratu_, heat2d_euler_, heat2d_midpoint_,
                       heat2d_trapezoid_, heat3d_euler_, heat3d_midpoint_, heat3d_trapezoid_)

__all__ = [
    "NKError", "device_count", "load", "EisenstatWalker", "Fixed", "Forcing", "JacobianOperator", "Result", "Stats",
    "mul_", "newton_krylov", "newton_krylov_", "newton_krylov_native", "transpose", "collect", "TransposeOperator", "Context", "DeviceArray", "Grid", "default_context",
    "set_default_context", "dist_unique_id", "init_distributed", "slab", "block", "G_Euler_", "G_Midpoint_", "G_Trapezoid_", "diffusion_", "diffusion3d_", "solve",
    "KrylovConstructor", "exp_", "kaxpby_", "kaxpy_", "kaxpy_norm_", "kcopy_", "kdivcopy_", "kdot", "kfill_", "knorm", "kref_",
    "DiagonalPreconditioner", "GmresPreconditioner", "Ilu0Preconditioner", "Preconditioner", "UserPreconditioner",
    "gmres_preconditioner", "ilu0",
    "jacobi", "jacobian_diag",
    "krylov_solve_", "krylov_workspace", "kscal_", "mgs_step_", "DeviceResidual", "UserResidual", "bc_zero_", "bratu2d_", "bratu_",
    "heat2d_euler_", "heat3d_euler_", "heat2d_midpoint_", "heat3d_midpoint_", "heat2d_trapezoid_", "heat3d_trapezoid_",
    "bc_periodic_",
]
