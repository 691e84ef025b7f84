"""Device context and grid functions (the device-side counterpart of `HaloVector`).

`examples/halovector.jl:1-45` wraps an (N+2) x (M+2) OffsetArray whose ghost layer holds the
boundary values and whose `length` is the interior count.  `DeviceArray` is the MI355X layout of
the same idea: the interior is one dense HBM array (x fastest, the reference's column-major
order), 256-byte aligned, with ONE ghost plane before and after it along the slowest axis.
Those ghost planes are zero (the physical Dirichlet boundary, `bc_zero!`) or, when the grid is
split over GPUs, the neighbouring slab's boundary plane written by the RCCL halo exchange.
Boundaries along the other axes are applied inside the kernels.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import check, load


class Context:
    """One GPU: a HIP stream, reduction scratch and (optionally) an RCCL communicator (nk_ctx)."""

    def __init__(self, device: int | None = None):
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        lib = load()
        h = C.c_void_p()
        rc = lib.nk_ctx_create(int(device), C.byref(h))
        if rc != 0:
            raise _lib.NKError(f"nk_ctx_create(device={device}) failed ({rc}): no usable MI355X visible -- "
                               "the HIP path has no CPU fallback")
        self.handle = h
        self.device = device
        self.rank, self.nranks = 0, 1

    def check(self, rc, what=""):
        check(rc, self.handle, what)

    def sync(self):
        self.check(load().nk_sync(self.handle), "nk_sync")

    @property
    def stream(self) -> int:
        """The library's hipStream_t (every kernel and every user-residual callback runs on it)."""
        return load().nk_ctx_stream(self.handle) or 0

    def torch_stream(self):
        """`with ctx.torch_stream(): ...` makes torch enqueue on the library's stream (for user residuals)."""
        import torch

        _lib.require_torch_first()
        return torch.cuda.stream(torch.cuda.ExternalStream(self.stream, device=torch.device("cuda", self.device)))

    def close(self):
        if getattr(self, "handle", None):
            load().nk_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- distribution ------------------------------------------------------------------------
    @property
    def mailbox_active(self) -> bool:
        return bool(load().nk_dist_mailbox_active(self.handle))

    def path_info(self) -> dict:
        """The distributed path this context runs (nk_dist_path): transport, resident sweep, in-launch
        ghost planes, ranks sharing the GPU, the device's PCI bus id."""
        info = _lib.nk_path_info()
        self.check(load().nk_dist_path(self.handle, C.byref(info)), "nk_dist_path")
        out = {name: getattr(info, name) for name, _ in _lib.nk_path_info._fields_}
        out["pci_bus_id"] = info.pci_bus_id.decode(errors="replace")
        out["mailbox_host"] = info.mailbox == 2  # the host shared-memory mailbox (nkhip.h nk_path_info)
        for k in ("rccl", "mailbox", "resident_sweep", "halo_in_launch", "mailbox_error"):
            out[k] = bool(out[k])
        return out

    def mailbox_handle(self) -> bytes:
        """64-byte IPC handle of this context's peer mailbox (nk_dist_mailbox_handle)."""
        buf = C.create_string_buffer(64)
        self.check(load().nk_dist_mailbox_handle(self.handle, buf), "nk_dist_mailbox_handle")
        return buf.raw

    def mailbox_open(self, rank: int, nranks: int, handles: bytes):
        """Reductions across `nranks` contexts through their mailboxes, without an RCCL communicator
        (nk_dist_mailbox_open; `handles` = the ranks' mailbox_handle() concatenated in rank order)."""
        if len(handles) != 64 * nranks:
            raise ValueError("handles must hold nranks x 64 bytes")
        self.check(load().nk_dist_mailbox_open(self.handle, rank, nranks, handles), "nk_dist_mailbox_open")
        self.rank, self.nranks = rank, nranks

    def set_process_grid(self, px: int, py: int, pz: int):
        """3D blocks instead of z-slabs (nk_dist_grid): px x py x pz ranks, rank = (iz py + iy) px + ix.
        Call after the ranks are connected and before allocating any vector: a 3D grid function then
        carries its x / y ghost faces too, exchanged with its z planes through the peer mailbox."""
        self.check(load().nk_dist_grid(self.handle, int(px), int(py), int(pz)), "nk_dist_grid")
        self.pgrid = (int(px), int(py), int(pz))

    def init_distributed(self, rank: int, nranks: int, unique_id: bytes):
        self.check(load().nk_dist_init(self.handle, rank, nranks, unique_id), "nk_dist_init")
        self.rank, self.nranks = rank, nranks

    # -- profiling ---------------------------------------------------------------------------
    def prof_enable(self, every: int = 1):
        """Time every `every`-th launch of each kernel class with HIP events (0 = off)."""
        self.check(load().nk_prof_enable(self.handle, int(every)), "nk_prof_enable")

    def prof_reset(self):
        self.check(load().nk_prof_reset(self.handle), "nk_prof_reset")

    def prof_read(self) -> dict:
        cap = 64
        buf = (_lib.nk_prof_entry * cap)()
        cnt = C.c_int32(0)
        self.check(load().nk_prof_read(self.handle, buf, cap, C.byref(cnt)), "nk_prof_read")
        return {buf[i].name.decode(): dict(launches=buf[i].launches, timed=buf[i].timed, ms=buf[i].total_ms,
                                           bytes=buf[i].bytes, bytes_all=buf[i].bytes_all,
                                           dram_all=buf[i].dram_bytes_all, kernel=buf[i].kernel.decode())
                for i in range(min(cnt.value, cap))}


_default_ctx: Context | None = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context()
    return _default_ctx


def set_default_context(ctx: Context):
    global _default_ctx
    _default_ctx = ctx


@dataclass(frozen=True)
class Grid:
    """Interior grid of one rank: local extents (x fastest) + the slab's place in the global grid."""
    shape_xyz: tuple          # local (nx,) / (nx, ny) / (nx, ny, nz)
    global_xyz: tuple         # global extents
    offset: int = 0           # first global index of this slab along the slowest axis
    origin: tuple = None      # 3D blocks: first global (x, y, z) index of this block (None: (0, 0, offset))

    @staticmethod
    def full(*dims) -> "Grid":
        return Grid(tuple(int(d) for d in dims), tuple(int(d) for d in dims), 0)

    @property
    def dim(self) -> int:
        return len(self.shape_xyz)

    @property
    def n(self) -> int:
        return int(np.prod(self.shape_xyz))

    @property
    def nxyz(self):
        s = tuple(self.shape_xyz) + (1,) * (3 - self.dim)
        return s[0], s[1], s[2]

    @property
    def np_shape(self):
        """numpy (C-order) shape with x fastest: (nx,), (ny, nx), (nz, ny, nx)."""
        return tuple(reversed(self.shape_xyz))

    def geometry_problem(self) -> _lib.nk_problem:
        """An nk_problem that carries only this grid's geometry (for allocation)."""
        nx, ny, nz = self.nxyz
        kind = {1: _lib.NK_BRATU1D, 2: _lib.NK_BRATU2D, 3: _lib.NK_HEAT3D_EULER}[self.dim]
        return _lib.nk_problem(kind, 0, nx, ny, nz, 1.0, 1.0, 1.0, 0.0, 0.0, 0.0, 1)


class DeviceArray:
    """A grid function in HBM: `similar`, `zero`, `copy`, `length` like HaloVector (halovector.jl:12-45)."""

    def __init__(self, grid: Grid, ctx: Context | None = None, *, _ptr=None):
        self.ctx = ctx or default_context()
        self.grid = grid
        if _ptr is None:
            p = C.c_void_p()
            gp = grid.geometry_problem()
            self.ctx.check(load().nk_vec_alloc(self.ctx.handle, C.byref(gp), C.byref(p)), "nk_vec_alloc")
            self.ptr = p.value
            self._owned = True
        else:
            self.ptr = _ptr
            self._owned = False

    # -- AbstractVector-ish protocol ---------------------------------------------------------
    def __len__(self):
        return self.grid.n

    @property
    def n(self) -> int:
        return self.grid.n

    @property
    def shape(self):
        return self.grid.np_shape

    def similar(self) -> "DeviceArray":
        return DeviceArray(self.grid, self.ctx)

    def zero(self) -> "DeviceArray":
        return DeviceArray(self.grid, self.ctx)  # nk_vec_alloc zero-fills, ghosts included

    def copy(self) -> "DeviceArray":
        out = DeviceArray(self.grid, self.ctx)
        self.ctx.check(load().nk_copy(self.ctx.handle, self.n, out.ptr, self.ptr), "nk_copy")
        return out

    def copyto_(self, src: "DeviceArray") -> "DeviceArray":
        self.ctx.check(load().nk_copy(self.ctx.handle, self.n, self.ptr, src.ptr), "nk_copy")
        return self

    def fill_(self, v: float) -> "DeviceArray":
        self.ctx.check(load().nk_fill(self.ctx.handle, self.n, self.ptr, float(v)), "nk_fill")
        return self

    # -- host transfer -----------------------------------------------------------------------
    @staticmethod
    def from_numpy(a, grid: Grid | None = None, ctx: Context | None = None) -> "DeviceArray":
        a = np.ascontiguousarray(a, dtype=np.float64)
        if grid is None:
            grid = Grid.full(*reversed(a.shape))
        if a.size != grid.n:
            raise ValueError(f"array of {a.size} elements does not fit grid {grid.shape_xyz}")
        d = DeviceArray(grid, ctx)
        d.ctx.check(load().nk_memcpy_h2d(d.ctx.handle, d.ptr, a.ctypes.data, a.size), "nk_memcpy_h2d")
        return d

    def torch(self, ghosts: bool = False):
        """Zero-copy torch view (numpy-order shape, x fastest) -- for user residuals.  ghosts=True
        includes the ghost plane on each side of the slowest axis (zero Dirichlet, or the neighbour
        slab's plane when distributed): shape (n_slow + 2, ...)."""
        import torch

        _lib.require_torch_first()
        shape, ptr = self.grid.np_shape, self.ptr
        if ghosts:
            plane = int(np.prod(shape[1:])) if len(shape) > 1 else 1
            shape, ptr = (shape[0] + 2,) + tuple(shape[1:]), self.ptr - 8 * plane
        view = type("_CAI", (), {})()
        view.__cuda_array_interface__ = {"shape": shape, "typestr": "<f8", "data": (ptr, False), "version": 3,
                                         "strides": None}
        return torch.as_tensor(view, device=torch.device("cuda", self.ctx.device))

    def to_numpy(self) -> np.ndarray:
        out = np.empty(self.grid.np_shape, dtype=np.float64)
        self.ctx.check(load().nk_memcpy_d2h(self.ctx.handle, out.ctypes.data, self.ptr, self.n), "nk_memcpy_d2h")
        return out

    def free(self):
        if self._owned and self.ptr and self.ctx.handle:
            load().nk_vec_free(self.ctx.handle, self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def __repr__(self):
        return f"DeviceArray(shape={self.shape}, device={self.ctx.device})"
