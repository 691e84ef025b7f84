"""In-process A/B of kernel variants (interleaved rounds, median reported).

Usage (GPU box): python tools/kbench.py [--n 16777216] [--rounds 5]
Not part of the product; drives the nkb_* hooks compiled into libnkhip_kbench.so.
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
ap.add_argument("--n", type=int, default=4096 * 4096)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--what", default="mgs,stencil")
ap.add_argument("--n3", type=int, default=512, help="3D stencil side (stencil3)")
ap.add_argument("--rows", default="8,16,32", help="stencil rows per tile")
ap.add_argument("--fast", default="0,2,4,6", help="stencil variant bits (launch_stencil_ex): 1 reciprocals, 4 VEC=4")
args = ap.parse_args()

ctx = ah.Context(0)
lib = ah.load()
lib.nkb_mgs_seq.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double)]
lib.nkb_copy.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.POINTER(C.c_double)]
lib.nkb_stencil3d.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double)]
lib.nkb_stencil.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                            C.POINTER(C.c_double)]
n = args.n
side = int(round(n ** 0.5))

MGS = {0: "U2", 1: "U2+nt(V_i)", 2: "U4+nt(V_i)", 3: "U2+nt(V_i,V_i+1)", 4: "U4+nt(V_i,V_i+1)",
       5: "U2+nt(V_i) chunked", 6: "U4+nt(V_i) chunked"}
configs = [("copy", None, None, None)]
if "mgs" in args.what:
    configs += [("mgs", v, alt, k) for k in (8, 16, 30) for v in MGS for alt in ((0, 1) if v in (5, 6) else (0,))]
ROWS = [int(x) for x in args.rows.split(",")]
FASTS = [int(x) for x in args.fast.split(",")]
ST = {(2, 2): ("jv_fd_dot", 40.0), (1, 2): ("jv_exact_dot", 32.0), (0, 1): ("residual_norm", 16.0)}
if "stencil" in args.what.replace("stencil3", ""):
    configs += [("st", mode_epi, rows, fast) for mode_epi in ST for rows in ROWS for fast in FASTS]
ST3 = {(2, 2): ("3d jv_fd_dot", 48.0), (0, 1): ("3d residual_norm", 24.0)}  # heat: + u_n
if "stencil3" in args.what:
    configs += [("st3", mode_epi, None, 0) for mode_epi in ST3]
res = {c: [] for c in configs}
for _ in range(args.rounds):
    for cfg in configs:
        us = C.c_double()
        if cfg[0] == "copy":
            rc = lib.nkb_copy(ctx.handle, n, args.reps, C.byref(us))
            nbytes = 16.0 * n
        elif cfg[0] == "st3":
            (mode, epi), fast = cfg[1], cfg[3]
            rc = lib.nkb_stencil3d(ctx.handle, args.n3, mode, epi, fast, args.reps, C.byref(us))
            nbytes = ST3[cfg[1]][1] * args.n3 ** 3
        elif cfg[0] == "st":
            (mode, epi), rows, fast = cfg[1], cfg[2], cfg[3]
            rc = lib.nkb_stencil(ctx.handle, side, side, mode, epi, rows, fast, args.reps, C.byref(us))
            nbytes = ST[cfg[1]][1] * side * side
        else:
            _, v, alt, k = cfg
            rc = lib.nkb_mgs_seq(ctx.handle, n, k, v, alt, 2, C.byref(us))
            nbytes = (32.0 * (k - 1) + 24.0) / k * n  # average algorithmic bytes per pass
        assert rc == 0, rc
        res[cfg].append((us.value, nbytes / (us.value * 1e-6) / 1e9))
for cfg, v in res.items():
    us = statistics.median(x[0] for x in v)
    gbs = statistics.median(x[1] for x in v)
    if cfg[0] == "copy":
        name = "copy (16 B/pt, 2 buffers)"
    elif cfg[0] == "st3":
        name = f"{ST3[cfg[1]][0]:>18s} tile rows= 4"
    elif cfg[0] == "st":
        name = f"{ST[cfg[1]][0]:>14s} rows={cfg[2]:2d} fast={cfg[3]}"
    else:
        name = f"mgs k={cfg[3]:2d} {MGS[cfg[1]]:>11s} alt={cfg[2]}"
    print(f"{name:40s} {us:9.2f} us/pass  {gbs:8.1f} GB/s  ({gbs / 8000 * 100:5.1f}% of 8 TB/s)")
