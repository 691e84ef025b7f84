#!/bin/bash
# 3D stencil tile order / march direction / chunk length (kbench env NK_ST3_ZALT, NK_ST_MINPLANES):
# 0 plane-major (round-2 order), 1 whole tile columns per XCD band + odd chunks marching down,
# 2 plane-major + odd chunks marching down, 3 chunk pairs at consecutive band positions + odd chunks
# marching down; 16 / 32 / 64-plane chunks.  Bitwise check of mode 3 and 2 first.  (profiles/r03/ab_zalt2.log)
set -e
cd "$(dirname "$0")/.."
for z in 2 3; do
  NK_ST3_ZALT=$z timeout -k 10 300 python -u tools/kbench_cmp.py --cases 4:200:37:2:2:288:65824,6:200:37:2:2:256:65792,4:200:20:2:2:288:65824,8:130:77:0:1:0:65536 || true
done
K="timeout -k 10 300 python -u tools/kbench_st.py --rounds 5 --reps 10 --rows 0 --kinds 6 --side 512 --modes 2:2 --fast 256"
K4="timeout -k 10 300 python -u tools/kbench_st.py --rounds 5 --reps 10 --rows 0 --kinds 4 --side 512 --modes 2:2,0:1 --fast 288"
K5="timeout -k 10 300 python -u tools/kbench_st.py --rounds 5 --reps 10 --rows 0 --kinds 4 --side 512 --nz 64 --modes 2:2 --fast 32"
for mp in 16 32 64; do
  for z in 0 1 2 3; do
    echo "== NK_ST_MINPLANES=$mp NK_ST3_ZALT=$z"
    NK_ST_MINPLANES=$mp NK_ST3_ZALT=$z $K
    NK_ST_MINPLANES=$mp NK_ST3_ZALT=$z $K4
    NK_ST_MINPLANES=$mp NK_ST3_ZALT=$z $K5
  done
done
