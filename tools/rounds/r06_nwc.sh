#!/bin/bash
# does the Infinity Cache keep a part of V_{i+1} for its re-read as the next pass's V_i?
# The resident sweep at 4096^2 (k = 30, 128 slots per block: 89 registers + 39 LDS) with the first w slots'
# V_{i+1} loaded with the default policy and the rest non-temporally (kbench NK_RES_NWC = w; V_i is always
# non-temporal).  One process per w (the knob is read once), two rounds, interleaved.
set -e -o pipefail
OUT=gpurun_out/r06_nwc
mkdir -p "$OUT"
for r in 1 2; do
  for w in 128 96 64 48 32 0; do
    echo "round $r NK_RES_NWC=$w" >> "$OUT/nwc.log"
    NK_RES_NWC=$w timeout -k 10 120 python -u tools/kbench_res.py --n 16777216 --ks 30 --rvs 1000 --reps 5 >> "$OUT/nwc.log" 2>&1
  done
done
echo done
