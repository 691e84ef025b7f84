"""In-process A/B of the x-update kernel (k_update_x<U>): U elements (16 B) per thread and iteration.

Usage (GPU box): python tools/kbench_upd.py [--n 67108864] [--rounds 5]
Not part of the product; drives the nkb_update_x hook compiled into libnkhip_kbench.so.
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
ap.add_argument("--n", type=int, default=8192 * 8192)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--ks", default="1,2,3,4,8,12,16,30")
ap.add_argument("--us", default="1,2,4")
args = ap.parse_args()
ctx = ah.Context(0)
lib = ah.load()
lib.nkb_update_x.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double)]
res = {}
for _ in range(args.rounds):
    for k in map(int, args.ks.split(",")):
        for u in map(int, args.us.split(",")):
            t = C.c_double()
            rc = lib.nkb_update_x(ctx.handle, args.n, k, u, args.reps, C.byref(t))
            assert rc == 0, rc
            res.setdefault((k, u), []).append(t.value)
print(f"k_update_x, n = {args.n}: median us per launch over {args.rounds} interleaved rounds (bytes = 8 n (k + 2))")
for (k, u), v in sorted(res.items()):
    us = statistics.median(v)
    print(f"k={k:3d} U={u}  {us:9.1f} us  {8.0 * args.n * (k + 2) / us / 1e3:7.1f} GB/s")
