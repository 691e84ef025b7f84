#!/bin/bash
# One-shot LDS tiles 256 columns wide (k_st2t<..., VEC 4>, kbench fast bit 131072 with 8192 = 8 rows /
# 16384 = 4 rows) vs the row march: bitwise check first, then timing (profiles/r03/ab_tile4.log)
set -e
cd "$(dirname "$0")/.."
[ -n "$SKIP_CMP" ] || timeout -k 10 300 python -u tools/kbench_cmp.py --cases 2:1000:1:2:2:0:139264,2:1000:1:2:2:0:147456,3:1000:1:0:1:0:139264,3:1000:1:2:2:288:139520,5:1000:1:2:2:256:139520 || true
K="timeout -k 10 300 python -u tools/kbench_st.py --rounds 7 --reps 10 --rows 0"
$K --kinds 2 --side 4096 --modes 2:2 --fast 0,139264
$K --kinds 2 --side 4096 --modes 2:0 --fast 0,139264,147456,8192
$K --kinds 3 --side 4096 --modes 0:1,2:2 --fast 0,139264
$K --kinds 3 --side 8192 --modes 0:0,2:0 --fast 0,139264,147456
