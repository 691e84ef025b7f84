#!/bin/bash
# short tiles in address order (one-shot streaming shape, fast bit 2048) vs marched 32-row tiles in
# XCD-contiguous bands: is the access shape what holds the stencils at ~0.65 of 8 TB/s?
set -e
cd "$(dirname "$0")/.."
K="timeout -k 10 300 python -u tools/kbench_st.py --rounds 5 --reps 10"
$K --kinds 3 --side 8192 --modes 0:0 --rows 1,2,4,8,32 --fast 0,2048
$K --kinds 2 --side 4096 --modes 2:0 --rows 1,2,4,8,32 --fast 0,2048
$K --kinds 7 --side 8192 --modes 2:0 --rows 1,2,4,8,32 --fast 160,2208
