"""A/B of the resident MGS sweep (one launch per Arnoldi step, q on chip) against the per-pass
chain of k_mgs_pass launches, on the same q and basis.  Not part of the product.

Usage (GPU box): python tools/kbench_res.py [--n 16777216] [--ks 8,16,30] [--rvs 0,16,32,48]
"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("NK_KBENCH_LIB", "1")  # the nkb_* hooks live in lib/libnkhip_kbench.so
import _nkpath  # noqa: F401,E402
import ariadne_hip as ah  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=4096 * 4096)
ap.add_argument("--ks", default="8,16,30")
ap.add_argument("--rvs", default="0,16,32,48")
ap.add_argument("--reps", type=int, default=5)
args = ap.parse_args()

ctx = ah.Context(0)
lib = ah.load()
lib.nkb_mgs_res.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double),
                            C.POINTER(C.c_double), C.POINTER(C.c_double)]
for k in [int(x) for x in args.ks.split(",")]:
    for rv in [int(x) for x in args.rvs.split(",")]:
        us, ref = C.c_double(), C.c_double()
        diff = (C.c_double * 4)()
        rc = lib.nkb_mgs_res(ctx.handle, args.n, k, rv, args.reps, C.byref(us), C.byref(ref), diff)
        if rc != 0:
            print(f"k={k} rv={rv}: rc={rc} {lib.nk_last_error(ctx.handle)}", flush=True)
            sys.exit(1)
        print(f"k={k:2d} rv={rv:2d}  resident {us.value:7.2f} us/pass   chain {ref.value:7.2f} us/pass   "
              f"speedup {ref.value / us.value:5.2f}x   q diff {diff[0]:.2e}  h diff {diff[1]:.2e}  (LDS slots {diff[2]:.0f}, {diff[3]:.0f} blocks)", flush=True)
