#!/bin/bash
# 3D stencils: whole tile columns per XCD band with odd z-chunks marching down (A.zalt = 1; run with
# NK_ST3_ZALT=1 -- the default was 1 when this log was taken, it is 0 now) vs the plane-major order (kbench fast bit 65536): bitwise check of out / V_k first, then timing
# (profiles/r03/ab_zalt.log).  The reductions differ in the last bits (another block -> tile map and
# accumulation order), every point value must not.
set -e
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u tools/kbench_cmp.py --cases 4:200:37:0:1:0:65536,4:200:37:2:2:288:65824,4:200:37:2:2:32:65568,6:200:37:2:2:256:65792,6:200:37:1:2:0:65536,8:200:37:2:2:256:65792,8:200:37:0:1:0:65536,4:130:64:2:2:288:65824,4:200:20:2:2:288:65824,6:96:20:2:2:256:65792 || true
K="timeout -k 10 300 python -u tools/kbench_st.py --rounds 5 --reps 10 --rows 0"
$K --kinds 4 --side 512 --modes 2:2 --fast 288,65824,32,65568
$K --kinds 4 --side 512 --modes 0:1 --fast 0,65536
$K --kinds 4 --side 512 --nz 64 --modes 2:2 --fast 32,65568,288,65824
$K --kinds 4 --side 512 --nz 64 --modes 0:1 --fast 0,65536
$K --kinds 6 --side 512 --modes 2:2,0:1 --fast 256,65792
$K --kinds 8 --side 512 --modes 2:2 --fast 256,65792
echo "== NK_ST_MINPLANES=32"
NK_ST_MINPLANES=32 $K --kinds 4 --side 512 --modes 2:2 --fast 288,65824
NK_ST_MINPLANES=32 $K --kinds 6 --side 512 --modes 2:2 --fast 256,65792
