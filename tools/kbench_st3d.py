"""In-process A/B of the 3D heat stencil's z-march length (planes per tile) -- k_st3d.

Every tile re-reads the two planes around its z-range, so a tile of P planes loads (P + 2) / P of
the compulsory bytes; longer marches cut that but leave fewer blocks.  Usage (GPU box):
    python tools/kbench_st3d.py [--n 512] [--nz 512,64] [--rounds 5]
Not part of the product; drives the nkb_stencil3d_ex hook compiled into libnkhip_kbench.so.
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
ap.add_argument("--n", type=int, default=512)
ap.add_argument("--nz", default="512,64")
ap.add_argument("--planes", default="0,8,16,32,64")
ap.add_argument("--variants", default="0", help="fast bits: 0 k_st3d (per-wave y loads), 8 k_st3l NW=4, 16 k_st3l NW=8")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=10)
args = ap.parse_args()
ctx = ah.Context(0)
lib = ah.load()
lib.nkb_stencil3d_ex.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                 C.c_int, C.POINTER(C.c_double)]
VNAME = {0: "st3d", 8: "st3l/4", 16: "st3l/8"}
# (kind, mode, epi) -> (label, words per point): mode 0 res / 2 FD; epi 1 sumsq, 2 dot (aux)
CASES = {(4, 2, 2): ("euler FD Jv + dot", 6), (4, 0, 1): ("euler residual + norm", 3),
         (6, 2, 2): ("midpoint FD Jv + dot", 6), (6, 0, 1): ("midpoint residual + norm", 3)}
res = {}
for _ in range(args.rounds):
    for nz in map(int, args.nz.split(",")):
        for case in CASES:
            for pl in map(int, args.planes.split(",")):
                for var in map(int, args.variants.split(",")):
                    if pl > nz:
                        continue
                    t = C.c_double()
                    rc = lib.nkb_stencil3d_ex(ctx.handle, args.n, nz, case[0], case[1], case[2], pl, var, args.reps,
                                              C.byref(t))
                    if rc != 0:  # e.g. more blocks than the reduction slots hold (short marches at 512^3)
                        continue
                    res.setdefault((nz, case, pl, var), []).append(t.value)
print(f"k_st3d at {args.n}^2 x nz: median us per launch over {args.rounds} rounds (GB/s on the compulsory bytes)")
for (nz, case, pl, var), v in sorted(res.items()):
    us = statistics.median(v)
    label, words = CASES[case]
    print(f"nz={nz:4d} {label:26s} {VNAME[var]:7s} planes={pl if pl else 'auto':>4}  {us:8.1f} us  "
          f"{8.0 * words * args.n * args.n * nz / us / 1e3:7.1f} GB/s")
