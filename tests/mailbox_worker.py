"""Worker for tests/test_hip_dist.py::test_mailbox_two_ranks_one_gpu (launched by torch.distributed.run).

Mailbox-only ranks (no RCCL communicator: both share device 0 on a one-GPU box, which RCCL refuses):
the ranks exchange their mailbox IPC handles over gloo, open each other's mailboxes, and every
reduction (kdot, knorm) then sums over ranks through the peer mailboxes.  Integer-valued data make
every sum exact, so the expected results are exact too.
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _nkpath  # noqa: F401,E402
import ariadne_hip as ah  # noqa: E402
import torch.distributed as dist  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--out", required=True)
args = ap.parse_args()
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
ctx = ah.Context(0)
ah.set_default_context(ctx)
handles = [None] * world
dist.all_gather_object(handles, ctx.mailbox_handle())
ctx.mailbox_open(rank, world, b"".join(handles))
results = []
n = 100_003  # odd: the tail element path too
for k in range(1, 40):
    x = ah.DeviceArray.from_numpy(np.full(n, float(rank + k)))
    y = ah.DeviceArray.from_numpy(np.arange(n, dtype=np.float64) % 7)
    results.append([ah.kdot(n, x, y), ah.knorm(n, y) ** 2])
dist.barrier()
if rank == 0:
    json.dump({"results": results, "world": world, "n": n}, open(args.out + ".json", "w"))
ctx.sync()
dist.destroy_process_group()
