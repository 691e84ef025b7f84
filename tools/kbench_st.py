"""In-process A/B of stencil launch geometries for any problem kind (nkb_stencil_kind hook).

Usage (GPU box): python tools/kbench_st.py [--kinds 3,5,7] [--side 8192] [--rows 0,16,32,64,128] [--fast 0,4]
Not part of the product.  GB/s on the compulsory bytes (the launcher's algorithmic count).
"""
import argparse
import ctypes as C
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("NK_KBENCH_LIB", "1")  # the nkb_* hooks live in lib/libnkhip_kbench.so
import _nkpath  # noqa: F401,E402
import ariadne_hip as ah  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--kinds", default="3,5,7")
ap.add_argument("--side", type=int, default=8192)
ap.add_argument("--nz", type=int, default=0, help="3D kinds: planes (default side)")
ap.add_argument("--ny", type=int, default=0, help="rows (default side)")
ap.add_argument("--modes", default="0:1,2:2", help="mode:epi pairs (0:1 residual+norm, 2:2 FD Jv+dot)")
ap.add_argument("--rows", default="0,16,32,64,128")
ap.add_argument("--fast", default="0,4", help="variant bits: 1 reciprocals for the divisions (not bit-faithful), "
                "4 VEC=4 (2D), 8/16 LDS tiles of 4/8 rows (3D), 32 F0 recomputed, 64 raw rows three ahead, "
                "128 bc_periodic!, 256 fused normalisation (V_k = v / h stored)")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=10)
args = ap.parse_args()
ctx = ah.Context(0)
lib = ah.load()
lib.nkb_stencil_kind.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int,
                                 C.c_int, C.c_int, C.POINTER(C.c_double)]
NAME = {2: "bratu2d", 3: "heat2d euler", 4: "heat3d euler", 5: "heat2d midpoint", 6: "heat3d midpoint",
        7: "heat2d trapezoid", 8: "heat3d trapezoid"}
MODE = {(0, 1): "residual+norm", (2, 2): "FD Jv+dot", (1, 2): "exact Jv+dot"}


def words(kind, mode, epi, fast=0):  # the launcher's algorithmic count (fast bit 32: F0 recomputed)
    heat = kind >= 3
    w = 1
    w += (1 + heat) if mode == 0 else ((1 + (not heat)) if mode == 1 else (3 + heat))
    f0r = mode == 2 and fast & 32 and (kind in (2, 3, 5, 7) or kind == 4)
    vout = mode != 0 and epi == 2 and fast & 256  # fused normalisation: V_k stored
    return w + (1 if epi == 2 else 0) - (1 if f0r else 0) + (1 if vout else 0)


res = {}
for _ in range(args.rounds):
    for kind in map(int, args.kinds.split(",")):
        dim3 = kind in (4, 6, 8)
        nz = (args.nz or args.side) if dim3 else 1
        for me in args.modes.split(","):
            mode, epi = map(int, me.split(":"))
            for rows in map(int, args.rows.split(",")):
                for fast in map(int, args.fast.split(",")):
                    t = C.c_double()
                    rc = lib.nkb_stencil_kind(ctx.handle, kind, args.side, args.ny or args.side, nz, mode, epi, rows, fast,
                                              args.reps, C.byref(t))
                    assert rc == 0, (kind, mode, epi, rows, fast, rc)
                    res.setdefault((kind, mode, epi, rows, fast, nz), []).append(t.value)
print(f"stencils at {args.side}^2 (x nz): median us per launch over {args.rounds} interleaved rounds")
for (kind, mode, epi, rows, fast, nz), v in res.items():
    us = statistics.median(v)
    gb = 8.0 * words(kind, mode, epi, fast) * args.side * (args.ny or args.side) * nz / us / 1e3
    print(f"{NAME[kind]:17s} {MODE.get((mode, epi), f'{mode}:{epi}'):14s} rows={rows:4d} fast={fast:2d}"
          f"  {us:9.1f} us  {gb:7.1f} GB/s  ({gb / 80:5.1f}% of 8 TB/s)")
