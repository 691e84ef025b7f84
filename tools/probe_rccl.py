"""Host-side cost of the scalar RCCL all-reduce (1-rank communicator, NK_DIST_FORCE=1) vs a plain
kernel launch: how fast can the host enqueue them, and how long does the GPU take."""
import ctypes as C
import os
import sys
import time

os.environ["NK_DIST_FORCE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _nkpath  # noqa: F401,E402
import numpy as np  # noqa: E402
import ariadne_hip as ah  # noqa: E402

ctx = ah.Context(0)
lib = ah.load()
x = ah.DeviceArray.from_numpy(np.ones(1024))
for label, dist in (("plain", False), ("rccl-1rank", True)):
    if dist:
        ctx.init_distributed(0, 1, ah.dist_unique_id())
    for what in ("allreduce", "scal"):
        if what == "allreduce" and not dist:
            continue
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(2000):
            if what == "allreduce":
                lib.nk_dist_allreduce_sum(ctx.handle, x.ptr, 1)
            else:
                lib.nk_scal(ctx.handle, 1024, 1.0, x.ptr)
        t1 = time.perf_counter()
        ctx.sync()
        t2 = time.perf_counter()
        print(f"{label:12s} {what:10s} host enqueue {1e6 * (t1 - t0) / 2000:7.2f} us/op, "
              f"total {1e6 * (t2 - t0) / 2000:7.2f} us/op")
