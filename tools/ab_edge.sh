#!/bin/bash
# x-edge loads issued by the edge lanes only (default) vs by every lane (fast bit 4096, round 2's form)
set -e
cd "$(dirname "$0")/.."
K="timeout -k 10 300 python -u tools/kbench_st.py --rounds 5 --reps 10 --rows 0"
$K --kinds 7 --side 8192 --modes 2:2,0:1 --fast 416,4512
$K --kinds 3 --side 8192 --modes 0:1,2:2 --fast 288,4384
$K --kinds 2 --side 4096 --modes 2:2 --fast 0,4096
$K --kinds 6 --side 512 --modes 0:1,2:2 --fast 256,4352
$K --kinds 4 --side 512 --nz 64 --modes 2:2 --fast 32,4128
