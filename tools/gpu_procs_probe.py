"""Which processes hold the GPU open during a torchrun multi-rank job (diagnostic for the box's
16-process guard).  Usage: python tools/gpu_procs_probe.py [--world 2] [--torch-first 1]"""
import argparse
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import os, sys, time
sys.path.insert(0, sys.argv[1])
import torch.distributed as dist
import _nkpath
import ariadne_hip as ah
ctx = ah.Context(0)
if sys.argv[2] == "1":  # as tests/dist_worker.py: gloo + the IPC mailbox
    dist.init_process_group("gloo")
    h = [None] * dist.get_world_size()
    dist.all_gather_object(h, ctx.mailbox_handle())
    ctx.mailbox_open(dist.get_rank(), dist.get_world_size(), b"".join(h))
time.sleep(float(sys.argv[3]))
'''


def holders():
    out = []
    for pid in os.listdir("/proc"):
        if not pid.isdigit():
            continue
        try:
            fds = os.listdir(f"/proc/{pid}/fd")
        except OSError:
            continue
        kfd = 0
        for fd in fds:
            try:
                t = os.readlink(f"/proc/{pid}/fd/{fd}")
            except OSError:
                continue
            if t == "/dev/kfd" or t.startswith("/dev/dri/"):
                kfd += 1
        if kfd:
            try:
                cmd = open(f"/proc/{pid}/cmdline").read().replace("\0", " ")[:120]
                ppid = open(f"/proc/{pid}/stat").read().split(")")[1].split()[1]
            except OSError:
                continue
            out.append((int(pid), int(ppid), kfd, cmd))
    return out


ap = argparse.ArgumentParser()
ap.add_argument("--world", type=int, default=2)
ap.add_argument("--mailbox", default="1")
args = ap.parse_args()
wf = "/tmp/gpu_probe_worker.py"
open(wf, "w").write(WORKER)
p = subprocess.Popen([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.world}",
                      "--master-addr", "127.0.0.1", "--master-port", "29613", wf, ROOT, args.mailbox, "12"])
time.sleep(9)
h = holders()
print(f"world={args.world}: {len(h)} processes hold /dev/kfd or /dev/dri", flush=True)
for pid, ppid, n, cmd in sorted(h):
    print(f"  pid {pid} ppid {ppid} fds {n}: {cmd}", flush=True)
print("rc", p.wait(timeout=120))
