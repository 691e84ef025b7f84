#!/bin/bash
# One-shot 8-row LDS tiles (k_st2t, kbench fast bit 8192) WITH the reduction epilogues, at sizes whose
# tile count fits one reduction slot (4096 x 4000: 16 000 tiles; 8192 x 2000: 16 000): is the 8 % the
# Bratu Jv gains without an epilogue there with its dot too?  (profiles/r03/ab_tile8.log)
set -e
cd "$(dirname "$0")/.."
K="timeout -k 10 300 python -u tools/kbench_st.py --rounds 7 --reps 10 --rows 0"
$K --kinds 2 --side 4096 --ny 4000 --modes 2:2,2:0 --fast 0,8192
$K --kinds 2 --side 4096 --ny 4000 --modes 2:2 --fast 288,8480
$K --kinds 3 --side 8192 --ny 2000 --modes 0:1,2:2 --fast 0,8192
$K --kinds 3 --side 8192 --ny 2000 --modes 2:2 --fast 288,8480
$K --kinds 7 --side 8192 --ny 2000 --modes 0:1,2:2 --fast 128,8320
