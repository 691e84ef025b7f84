"""Run the smoke path with torch imported first (as bench.py does for N > 1) and report which HIP
runtime / RCCL libraries the process actually mapped."""
import os
import sys

import torch  # noqa: F401  (loads torch's bundled libamdhip64 / librccl first)
import torch.distributed  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402

__graft_entry__.smoke()
libs = sorted({l.split()[-1] for l in open("/proc/self/maps") if ("amdhip64" in l or "rccl" in l or "nkhip" in l)})
print("mapped:", *libs, sep="\n  ")
