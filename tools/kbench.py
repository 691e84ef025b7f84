"""In-process A/B of kernel variants (interleaved rounds, median reported).

Usage (GPU box): python tools/kbench.py [--n 16777216] [--rounds 5]
Not part of the product; drives the nkb_* hooks compiled into libnkhip.so.
"""
import argparse
import ctypes as C
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _nkpath  # noqa: F401,E402
import ariadne_hip as ah  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=4096 * 4096)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=20)
args = ap.parse_args()

ctx = ah.Context(0)
lib = ah.load()
lib.nkb_mgs.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double)]
lib.nkb_copy.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.POINTER(C.c_double)]
n = args.n

MGS = {0: "U1", 1: "U2", 2: "U4", 3: "U2+nt(V_i)", 4: "U4+nt(V_i)", 5: "U2 last-pass", 6: "U8"}
configs = [("copy", None, None)] + [("mgs", v, g) for v in MGS for g in (1024, 2048, 4096)]
res = {c: [] for c in configs}
for _ in range(args.rounds):
    for cfg in configs:
        us = C.c_double()
        if cfg[0] == "copy":
            rc = lib.nkb_copy(ctx.handle, n, args.reps, C.byref(us))
            nbytes = 16.0 * n
        else:
            rc = lib.nkb_mgs(ctx.handle, n, cfg[1], cfg[2], args.reps, C.byref(us))
            nbytes = (32.0 if cfg[1] != 5 else 24.0) * n
        assert rc == 0, rc
        res[cfg].append((us.value, nbytes / (us.value * 1e-6) / 1e9))
for cfg, v in res.items():
    us = statistics.median(x[0] for x in v)
    gbs = statistics.median(x[1] for x in v)
    name = "copy (16 B/pt)" if cfg[0] == "copy" else f"mgs {MGS[cfg[1]]:>14s} grid={cfg[2]}"
    print(f"{name:40s} {us:9.2f} us  {gbs:8.1f} GB/s  ({gbs / 8000 * 100:5.1f}% of 8 TB/s)")
