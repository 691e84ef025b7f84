"""Run one kernel configuration a few times (for rocprofv3 --pmc): FD Jv (2D Bratu 4096^2) and an MGS sweep."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("NK_KBENCH_LIB", "1")  # the nkb_* hooks live in lib/libnkhip_kbench.so
import _nkpath  # noqa: F401,E402
import ariadne_hip as ah  # noqa: E402

ctx = ah.Context(0)
lib = ah.load()
lib.nkb_stencil.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                            C.POINTER(C.c_double)]
lib.nkb_mgs_seq.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double)]
us = C.c_double()
what = sys.argv[1] if len(sys.argv) > 1 else "both"
if what in ("both", "jv"):
    assert lib.nkb_stencil(ctx.handle, 4096, 4096, 2, 2, 16, 0, 5, C.byref(us)) == 0
    print("jv_fd_dot us", us.value)
if what in ("both", "mgs"):
    assert lib.nkb_mgs_seq(ctx.handle, 4096 * 4096, 8, 1, 0, 1, C.byref(us)) == 0
    print("mgs us/pass", us.value)
