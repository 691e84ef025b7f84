"""The FD Jv's stream pattern without its arithmetic: 4 reads + 1 write per point (nkb_stream_jv in
libnkhip_kbench.so), against the plain copy (nkb_copy), at the Jv's own size (4096^2: 134 MB per
vector, 671 MB per pass) and at 1 GiB vectors.  Answers DESIGN §8's question: how much of the 2D
march's ~115 us floor (without any exp) is the access pattern itself.

Usage (GPU box): python tools/stream_jv.py [--rounds 3]
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
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--reps", type=int, default=20)
args = ap.parse_args()
ctx = ah.Context(0)
lib = ah.load()
for f in (lib.nkb_stream_jv,):
    f.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double)]
lib.nkb_copy.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.POINTER(C.c_double)]
NAMES = {0: "4R1W U1 grid-stride", 1: "4R1W U2 grid-stride", 2: "4R1W U2 chunk", 3: "4R1W U4 chunk"}
us = C.c_double()
for n in (4096 * 4096, 1 << 27):  # the Jv's own size; 1 GiB vectors
    rows = {}
    for _ in range(args.rounds):
        assert lib.nkb_copy(ctx.handle, n, args.reps, C.byref(us)) == 0
        rows.setdefault(("copy 1R1W", 0), []).append(us.value)
        for v in NAMES:
            for g in (1024, 2048, 4096, 8192, 32768):
                assert lib.nkb_stream_jv(ctx.handle, n, v, g, args.reps, C.byref(us)) == 0
                rows.setdefault((NAMES[v], g), []).append(us.value)
    print(f"n = {n} doubles per vector")
    for (name, g), t in rows.items():
        m = statistics.median(t)
        b = (16.0 if name.startswith("copy") else 40.0) * n
        print(f"  {name:22s} grid {g:6d}  {m:9.1f} us  {b / m / 1e3:7.1f} GB/s", flush=True)
