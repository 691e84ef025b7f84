#!/bin/bash
# stencil tile height vs row-stride camping: power-of-two row bands march in lock-step over addresses
# a power of two apart (profiles/r03/ab_rows.log)
set -e
cd "$(dirname "$0")/.."
K="timeout -k 10 300 python -u tools/kbench_st.py --rounds 5 --reps 10"
$K --kinds 3 --side 8192 --modes 0:1 --rows 16,24,31,32,33,40,48,64 --fast 0
$K --kinds 7 --side 8192 --modes 2:2 --rows 16,24,31,32,33,40,48 --fast 416
$K --kinds 2 --side 4096 --modes 2:2 --rows 16,24,31,32,33,40 --fast 0
$K --kinds 6 --side 512 --modes 0:1 --rows 8,12,15,16,17,24,32 --fast 0
$K --kinds 4 --side 512 --nz 64 --modes 2:2 --rows 8,12,15,16,21,32,64 --fast 32
