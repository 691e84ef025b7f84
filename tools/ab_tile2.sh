#!/bin/bash
# 2D one-shot LDS tiles (k_st2t, fast bits 8192 / 16384 / 32768 = 8 / 4 / 16 rows) vs the march:
# bitwise check first, then timing (profiles/r03/ab_tile2.log)
set -e
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u tools/kbench_cmp.py --cases 3:1000:1:0:1:0:8192,3:1000:1:2:2:288:8480,7:1000:1:2:2:416:8608,7:1000:1:0:1:128:8320,5:1000:1:2:2:288:8480,2:1000:1:2:2:0:8192,2:1000:1:1:2:0:32768,7:1000:1:1:2:384:16768,3:1000:1:2:3:0:8192
K="timeout -k 10 300 python -u tools/kbench_st.py --rounds 5 --reps 10 --rows 0"
$K --kinds 3 --side 8192 --modes 0:0 --fast 0,8192,16384,32768
$K --kinds 3 --side 8192 --modes 2:0 --fast 288,8480,16672,33056
$K --kinds 7 --side 8192 --modes 2:0 --fast 160,8352,16544,32928
$K --kinds 2 --side 4096 --modes 2:0 --fast 0,8192,16384,32768
$K --kinds 2 --side 4096 --modes 2:2 --fast 0,32768
$K --kinds 3 --side 4096 --modes 0:1 --fast 0,32768
