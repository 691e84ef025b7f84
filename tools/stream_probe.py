"""HBM streaming-rate probe (copy kernel variants x grid sizes), drives nkb_stream in libnkhip_kbench.so.

Usage (GPU box): python tools/stream_probe.py [--n 134217728] [--rounds 3]
Vectors of n doubles (default 1 GiB each: far beyond the 256 MB Infinity Cache).
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
ap.add_argument("--n", type=int, default=1 << 27)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--reps", type=int, default=10)
args = ap.parse_args()
ctx = ah.Context(0)
lib = ah.load()
lib.nkb_stream.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double)]
NAMES = {0: "copy U1 gs", 1: "copy U2 gs", 2: "copy U4 gs", 3: "copy U2 chunk", 4: "copy U4 chunk",
         5: "copy U2 gs-blk", 6: "copy U4 gs-blk", 7: "mgs U1 gs", 8: "mgs U2 gs", 9: "mgs U2 chunk",
         10: "mgs U4 chunk", 11: "mgs U2 gs-blk", 12: "mgs U4 gs-blk", 13: "mgs U1 chunk",
         14: "copy U1 gs ntl", 15: "copy U1 gs ntl+nts", 16: "copy U1 gs nts", 17: "copy U4 chunk ntl+nts",
         18: "copy U2 gs ntl+nts"}
BYTES = {v: (16.0 if (v < 7 or v >= 14) else 32.0) for v in NAMES}
ap2 = [int(x) for x in os.environ.get("NK_PROBE_VARIANTS", ",".join(map(str, NAMES))).split(",")]
grids = [int(x) for x in os.environ.get("NK_PROBE_GRIDS", "512,1024,1536,2048,4096,8192,32768").split(",")]
configs = [(v, g) for v in ap2 for g in grids]
res = {k: [] for k in configs}
us = C.c_double()
for _ in range(args.rounds):
    for v, g in configs:
        assert lib.nkb_stream(ctx.handle, args.n, v, g, args.reps, C.byref(us)) == 0
        res[(v, g)].append(us.value)
for (v, g), t in res.items():
    m = statistics.median(t)
    gbs = BYTES[v] * args.n / (m * 1e-6) / 1e9
    print(f"{NAMES[v]:16s} grid={g:>6} {m:9.1f} us  {gbs:7.0f} GB/s ({gbs / 80:5.1f}% of 8 TB/s)")
