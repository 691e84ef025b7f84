"""In-process A/B of the 3D stencils' y-march (k_st3y, fast bit 2^19) against the z-march (k_st3l), on
config 5's slab (512^2 x 64) and the whole 512^3 grid.  The y-march's rows per chunk come from
NK_ST3Y_ROWS (read once per process: run the tool once per value).  Usage (GPU box):
    NK_ST3Y_ROWS=64 python tools/kbench_ym.py [--nz 64,512] [--rounds 5]
Not part of the product; drives nkb_stencil3d_ex of libnkhip_kbench.so.
"""
import argparse
import ctypes as C
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("NK_KBENCH_LIB", "1")
import _nkpath  # noqa: F401,E402
import ariadne_hip as ah  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=512)
ap.add_argument("--nz", default="64,512")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=10)
args = ap.parse_args()
ctx = ah.Context(0)
lib = ah.load()
lib.nkb_stencil3d_ex.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                 C.c_int, C.POINTER(C.c_double)]
YM = 1 << 19
VARS = {8: "z-march NW4", 16: "z-march NW8", YM | 8: "y-march NW4", YM | 16: "y-march NW8"}
CASES = {(4, 2, 2): ("euler FD Jv + dot", 6), (4, 0, 1): ("euler residual + norm", 3),
         (6, 2, 2): ("midpoint FD Jv + dot", 6), (6, 0, 1): ("midpoint residual + norm", 3),
         (8, 2, 2): ("trapezoid FD Jv + dot", 6)}
res = {}
for _ in range(args.rounds):
    for nz in map(int, args.nz.split(",")):
        for case in CASES:
            for var in VARS:
                t = C.c_double()
                rc = lib.nkb_stencil3d_ex(ctx.handle, args.n, nz, case[0], case[1], case[2], 0, var, args.reps, C.byref(t))
                if rc != 0:
                    continue
                res.setdefault((nz, case, var), []).append(t.value)
rows = os.environ.get("NK_ST3Y_ROWS", "64")
print(f"3D stencils at {args.n}^2 x nz, y-march rows per chunk {rows}: median us per launch over {args.rounds} rounds "
      f"(GB/s on the compulsory bytes, fraction of 8 TB/s)")
for (nz, case, var), v in sorted(res.items()):
    us = statistics.median(v)
    label, words = CASES[case]
    gbs = words * 8.0 * args.n * args.n * nz / (us * 1e-6) / 1e9
    print(f"nz={nz:4d} {label:26s} {VARS[var]:12s} {us:9.1f} us  {gbs:7.0f} GB/s  {gbs / 8000:.3f}", flush=True)
