"""VGPR / AGPR / scratch of every kernel in a built object (the code object's metadata notes).
usage: python tools/vgprs.py newtonkrylov.jl_amd/build/nk_st_7.o [substring of the demangled name ...]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
obj, pats = sys.argv[1], sys.argv[2:]
with tempfile.TemporaryDirectory() as t:
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={t}/fat.bin", obj], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={t}/fat.bin",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={t}/k.co"], check=True)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", f"{t}/k.co"], check=True, capture_output=True,
                           text=True).stdout
kernels = []
cur = None
for line in notes.splitlines():
    if re.match(r"^  - \.", line):  # a new kernel record (args are indented deeper)
        cur = {}
        kernels.append(cur)
    m = re.match(r"^  (?:- |  )\.(\w+):\s+(\S+)", line)
    if m and cur is not None:
        cur[m.group(1)] = m.group(2)
kernels = [k for k in kernels if k.get("name")]
names = subprocess.run(["c++filt"], input="\n".join(k["name"] for k in kernels), capture_output=True,
                       text=True).stdout.splitlines()
for k, n in zip(kernels, names):
    if pats and not any(p in n for p in pats):
        continue
    print(f"vgpr {k.get('vgpr_count','?'):>4} agpr {k.get('agpr_count','?'):>3} scratch "
          f"{k.get('private_segment_fixed_size','?'):>4} lds {k.get('group_segment_fixed_size','?'):>6}  "
          f"{n.replace('(nk::KArgs)', '').replace('nk::(anonymous namespace)::', '')}")
