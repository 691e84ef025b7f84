"""Bitwise check of stencil variants against the default kernel (nkb_stencil_cmp, kbench build):
out, the stored V_k and the reduction of variant B against variant A on the same pseudo-random operands.
Usage (GPU box): python tools/kbench_cmp.py --cases "3:8192:1:0:1:0:8192,..."  (kind:nx:nz:mode:epi:fa:fb)"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("NK_KBENCH_LIB", "1")
import _nkpath  # noqa: F401,E402
import ariadne_hip as ah  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cases", required=True)
args = ap.parse_args()
ctx = ah.Context(0)
lib = ah.load()
lib.nkb_stencil_cmp.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int,
                                C.c_int, C.POINTER(C.c_double)]
bad = 0
for case in args.cases.split(","):
    kind, nx, nz, mode, epi, fa, fb = map(int, case.split(":"))
    d = (C.c_double * 5)()
    ny = nx if nz == 1 or kind in (2, 3, 5, 7) else nx
    rc = lib.nkb_stencil_cmp(ctx.handle, kind, nx, ny - (3 if nx > 64 else 0), nz, mode, epi, fa, fb, d)
    assert rc == 0, (case, rc)
    same = d[0] == 0.0 and d[1] == 0.0 and d[2] == d[3]
    bad += not same
    print(f"{case:32s} out {d[0]:.3e} (max |out| {d[4]:.3e}) vk {d[1]:.3e} red {d[2]!r} vs {d[3]!r} "
          f"{'BITWISE' if same else 'DIFFERENT'}", flush=True)
print("all bitwise" if not bad else f"{bad} case(s) differ")
