#!/bin/bash
# does the stencils' fp64 division cost show? reciprocal variant (fast bit 1, not bit-faithful) vs the
# IEEE division on the kernel classes VERDICT r02 names (profiles/r03/ab_div.log)
set -e
cd "$(dirname "$0")/.."
K="timeout -k 10 300 python -u tools/kbench_st.py --rounds 5 --reps 10 --rows 0"
$K --kinds 7 --side 8192 --modes 2:2 --fast 416,417
$K --kinds 7 --side 8192 --modes 0:1 --fast 128,129
$K --kinds 3 --side 8192 --modes 2:2,0:1 --fast 0,1,288,289
$K --kinds 6 --side 512 --modes 0:1,2:2 --fast 0,1,256,257
$K --kinds 4 --side 512 --nz 64 --modes 2:2 --fast 32,33
$K --kinds 2 --side 4096 --modes 2:2 --fast 0,1
