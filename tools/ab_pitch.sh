#!/bin/bash
# Row pitch probe: the same stencils on grids whose rows are 28 / 32 / 36 KB (and 60 / 64 / 68 KB) long,
# the row count fixed, every row a whole number of 512-column tiles -- does a power-of-two row pitch
# (all concurrent tiles of a march at one address phase) cost bandwidth?  (profiles/r03/ab_pitch.log)
set -e
cd "$(dirname "$0")/.."
for ny in 4096 8192; do
  for side in $((ny - 512)) $ny $((ny + 512)); do
    timeout -k 10 240 python -u tools/kbench_st.py --kinds 2,3,7 --side $side --ny $ny --modes 0:1,2:2 --rows 0 \
      --fast 0 --rounds 3 --reps 10
  done
done
